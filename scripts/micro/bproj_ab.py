#!/usr/bin/env python3
"""bproj_fwd ([250, 100, 5] x [5, 8192] + z rows -> 819 MB fp32, nontemporal
stores) timed alone (events around the one launch): into a fresh buffer, into
the same buffer again, after a 410 MB nontemporal write elsewhere (the
encoder input projection that precedes it in the training step), and into
memory that such a write just left dirty (its freed block re-used)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from sketch_rnn_amd.utils import native  # noqa: E402

T, B, IN, G = 250, 100, 5, 8192
lib = native.require_hip().lib
x = torch.randn(T, B, IN, device="cuda")
W = torch.randn(IN, G, device="cuda")
zw = torch.randn(B, G, device="cuda")
xe = torch.randn(T, B, IN, device="cuda")
We = torch.randn(2, IN, 2048, device="cuda")
ln = torch.full((B,), T, dtype=torch.int64, device="cuda")
st = lambda: torch.cuda.current_stream().cuda_stream   # noqa: E731


def bproj(o):
    assert lib.skr_bproj_fwd(x.data_ptr(), W.data_ptr(), zw.data_ptr(), o.data_ptr(), T, B, IN, G, 0, st()) == 0


def inproj(o):   # 410 MB nontemporal write, [T, 2B, 2048]
    assert lib.skr_inproj_fwd(xe.data_ptr(), ln.data_ptr(), We.data_ptr(), None, o.data_ptr(), T, B, IN, 2048, st()) == 0


def t_one(pre, mk_out, reps=5):
    best = 1e9
    for _ in range(reps):
        o = pre()
        out = mk_out(o)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        bproj(out)
        ev[1].record()
        torch.cuda.synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]) * 1e3)
        del o, out
    return round(best, 1)


fixed = torch.empty(T, B, G, device="cuda")
res = {
    "same_buffer": t_one(lambda: None, lambda o: fixed),
    "fresh": t_one(lambda: None, lambda o: torch.empty(T, B, G, device="cuda")),
}
xp_keep = torch.empty(T, 2 * B, 2048, device="cuda")
res["after_inproj_write"] = t_one(lambda: inproj(xp_keep), lambda o: fixed)


best = 1e9
for _ in range(5):   # the 410 MB block written, freed, and bproj's output allocated over it
    t = torch.empty(T, 2 * B, 2048, device="cuda")
    inproj(t)
    del t
    out = torch.empty(T, B, G, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    bproj(out)
    ev[1].record()
    torch.cuda.synchronize()
    best = min(best, ev[0].elapsed_time(ev[1]) * 1e3)
    del out
res["into_freed_dirty_block"] = round(best, 1)
print(json.dumps(res), flush=True)
