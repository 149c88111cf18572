#!/usr/bin/env python3
"""bproj_fwd ([250, 100, 5] x [5, 8192] + z rows -> 819 MB fp32, nontemporal
stores) timed in isolation: fresh output each call, the same output buffer
re-used, and an output buffer dirtied by a fill just before (is the write
rate sensitive to what the destination pages last held?)."""
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
out = torch.empty(T, B, G, device="cuda")
st = lambda: torch.cuda.current_stream().cuda_stream   # noqa: E731


def run(o):
    assert lib.skr_bproj_fwd(x.data_ptr(), W.data_ptr(), zw.data_ptr(), o.data_ptr(), T, B, IN, G, st()) == 0


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    best = 1e9
    for _ in range(reps):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        best = min(best, ev[0].elapsed_time(ev[1]) * 1e3)
    return best


res = {"same_buffer_us": timed(lambda: run(out)),
       "fresh_alloc_us": timed(lambda: run(torch.empty(T, B, G, device="cuda")))}
res["after_fill_us"] = min(timed(lambda: (out.fill_(1.0), torch.cuda.synchronize(), run(out))) for _ in range(1))
print(json.dumps({k: round(v, 1) for k, v in res.items()}), flush=True)
