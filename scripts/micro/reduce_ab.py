#!/usr/bin/env python3
"""Kernel-level A/B of the step's two streaming reductions at the vae_large
shapes (T*B = 25,000 rows, bf16 saves), CUDA-event timed, arms alternated:

* ``colsum``: the four LayerNorm gamma / beta reductions of the HyperLSTM
  backward (ops.reduce.colsum_many) at 4 vs 8 columns per thread;
* ``bproj``: the stroke-projection reductions of dXH [T, B, 8192] and
  dR_hyp [T, B, 1024] (ops.inproj.bproj_reduce), narrow vs wide kernel.

usage: reduce_ab.py [reps]   -- one JSON line per (kernel, arm)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.ops import inproj, reduce  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1e3 * a.elapsed_time(b) / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    ops.set_backend("hip")
    T, B, H, Hh, bf = 250, 100, 2048, 256, torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    rnd = lambda *s: torch.randn(*s, device="cuda", generator=g).to(bf)  # noqa: E731
    lnp = [(rnd(T * B, n), rnd(T * B, n)) for n in (4 * H, H, 4 * Hh, Hh)]
    x = torch.randn(T, B, 5, device="cuda", generator=g)
    dXH, dRY = rnd(T, B, 4 * H), rnd(T, B, 4 * Hh)
    res = {}
    for rep in range(3):
        for nc in (4, 8):
            reduce.COLSUM_NC = nc
            res.setdefault(("colsum", nc), []).append(timed(lambda: reduce.colsum_many(lnp), reps))
        for wide in (False, True):
            inproj.BPROJ_WIDE = wide
            res.setdefault(("bproj_dXH", wide), []).append(timed(lambda: inproj.bproj_reduce(x, dXH, raw=True), reps))
            res.setdefault(("bproj_dRY", wide), []).append(timed(lambda: inproj.bproj_reduce(x, dRY, raw=True), reps))
    for (k, arm), v in res.items():
        print(json.dumps({"kernel": k, "arm": arm, "us": [round(t, 1) for t in v], "min_us": round(min(v), 1)}))


if __name__ == "__main__":
    main()
