#!/usr/bin/env python3
"""Microbenchmark: skinny split-K GEMM vs hipBLASLt on the recurrent shapes."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from sketch_rnn_amd.ops import gemm  # noqa: E402

SHAPES = [  # (name, M, N, K, nd): the per-step products of the vae_large step
    ("R_main fwd", 100, 8192, 2048, 1),
    ("R_hyp  fwd", 100, 1024, 2304, 1),
    ("VEC    fwd", 100, 24576, 256, 1),
    ("DAM    bwd", 100, 2048, 8192, 1),
    ("DHZ    bwd", 100, 256, 24576, 1),
    ("DAY    bwd", 100, 2304, 1024, 1),
    ("enc    fwd", 100, 2048, 512, 2),
    ("enc    bwd", 100, 512, 2048, 2),
]


def timeit(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    dev = "cuda"
    for name, M, N, K, nd in SHAPES:
        a = torch.randn(nd * M, K, device=dev).to(torch.bfloat16)
        bt = torch.randn(nd, N, K, device=dev).to(torch.bfloat16)
        b = bt.transpose(1, 2).contiguous()
        res = []
        for algo in ("v1", "v2"):
          gemm.GEMM_ALGO = algo
          res.append(algo + ":")
          for bn in (64, 128):
            for S in sorted({gemm.plan_splits(M, N, K, nd), 1, 2, 4, 8, 16, 32}):
                if S < 1 or (K // 64) % S or N % bn:
                    continue
                out = torch.empty(S, nd * M, N, device=dev)
                us = timeit(lambda: gemm.rec_gemm(a, bt if nd > 1 else bt[0], out, S, nd, bn))
                if algo == "v2" and bn == 64:
                    ref = (a.float().view(nd, M, K) @ bt.float().transpose(1, 2)).reshape(nd * M, N)
                    err = (out.sum(0) - ref).abs().max().item()
                    assert err < 1e-2 * ref.abs().max().item() + 1e-3, (name, S, err)
                res.append("b%d/S%d %.1f" % (bn, S, us))
        out1 = torch.empty(nd, M, N, device=dev)
        if nd == 1:
            us_lib = timeit(lambda: torch.mm(a, b[0], out_dtype=torch.float32, out=out1[0]))
        else:
            us_lib = timeit(lambda: torch.bmm(a.view(nd, M, K), b, out_dtype=torch.float32, out=out1))
        flops = 2.0 * nd * M * N * K
        print("%s M=%d N=%d K=%d nd=%d  hipBLASLt %.1fus | %s | plan S=%d | %.1f GFLOP" % (
            name, M, N, K, nd, us_lib, " ".join(res), gemm.plan_splits(M, N, K, nd), flops / 1e9), flush=True)


if __name__ == "__main__":
    main()
