#!/usr/bin/env python3
"""Wide-batch decode GEMM shapes (B = 1024 rows, vae_large): hipBLASLt bf16
(torch.mm, fp32 out, a yardstick only) and the skinny split-K kernel run as 8
row blocks (csrc/skinny_gemm.hip). Prints one JSON line per (shape, impl)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    from sketch_rnn_amd.ops import gemm
    dev = "cuda"
    for (M, K, N) in [(1024, 2048, 8192), (1024, 2304, 1024), (1024, 2048, 128), (1024, 256, 24576),
                      (128, 2048, 8192)]:
        a = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(K, N, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev)
        us = timed(lambda: torch.mm(a, w, out_dtype=torch.float32, out=out))
        fl = 2 * M * N * K
        print(json.dumps({"M": M, "K": K, "N": N, "impl": "hipblaslt_bf16", "us": round(us, 2),
                          "tflops": round(fl / us / 1e6, 1)}), flush=True)
        if gemm.row_blocks(M) and N % 64 == 0:
            bt = w.t().contiguous()
            S = gemm.plan_splits(M, N, K, 1, torch.bfloat16)
            slabs = torch.empty(S, M, N, device=dev)
            try:
                usk = timed(lambda: gemm.rec_gemm(a, bt, slabs, S))
                print(json.dumps({"M": M, "K": K, "N": N, "impl": "skinny_rowblocks", "splits": S, "us": round(usk, 2),
                                  "tflops": round(fl / usk / 1e6, 1)}), flush=True)
            except Exception as e:   # noqa: BLE001
                print(json.dumps({"M": M, "K": K, "N": N, "impl": "skinny_rowblocks", "error": str(e)[:200]}),
                      flush=True)


if __name__ == "__main__":
    main()
