#!/usr/bin/env python3
"""Probe what bounds the skinny split-K GEMM on the vae_large per-step
shapes: time vs rows M (the activation operand re-read by every N tile) and
vs split-K S, as HIP-graph replays of back-to-back launches (each time
includes one kernel boundary). Output: one JSON line per (shape, M, S)."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from sketch_rnn_amd.ops import gemm  # noqa: E402

SHAPES = [("R_main", 8192, 2048), ("DAM", 2048, 8192), ("R_hyp", 1024, 2304), ("DAY", 2304, 1024),
          ("DHZ", 256, 24576)]


def timeit(fn, reps=100):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / reps * 1e6)
    return best


def main():
    dev = "cuda"
    for name, N, K in SHAPES:
        bt = torch.randn(N, K, device=dev).to(torch.bfloat16)
        for M in (16, 64, 100, 128):
            a = torch.randn(M, K, device=dev).to(torch.bfloat16)
            for S in (1, 2, 4, 8, 16, 32):
                if (K // 64) % S or (N // 64) * S > 1024:
                    continue
                out = torch.empty(S, M, N, device=dev)
                us = timeit(lambda: gemm.rec_gemm(a, bt, out, S))
                print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "S": S, "wg": (N // 64) * S,
                                  "us": round(us, 2)}), flush=True)


if __name__ == "__main__":
    main()
