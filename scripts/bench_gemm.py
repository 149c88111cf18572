#!/usr/bin/env python3
"""Microbenchmark: skinny split-K GEMM (v2 LDS-DMA ring) on the per-step
recurrent shapes of the vae_large step, swept over ring depth (NS), N-tile
width and split-K, plus the grouped launches the HyperLSTM uses, against
hipBLASLt. Times are HIP-graph replays of 200 back-to-back launches (so each
includes one kernel boundary)."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from sketch_rnn_amd.ops import gemm  # noqa: E402
from sketch_rnn_amd.utils import native  # noqa: E402

SHAPES = [  # (name, M, N, K, nd): the per-step products of the vae_large step
    ("R_main fwd", 100, 8192, 2048, 1),
    ("R_hyp  fwd", 100, 1024, 2304, 1),
    ("VEC    fwd", 100, 24576, 256, 1),
    ("DAM    bwd", 100, 2048, 8192, 1),
    ("DHZ    bwd", 100, 256, 24576, 1),
    ("DAY    bwd", 100, 2304, 1024, 1),
]
GROUPS = [("R_main+R_hyp", 0, 1), ("DAM+DHZ", 3, 4)]


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
    lib = native.require_hip().lib
    ops = {}
    for name, M, N, K, nd in SHAPES:
        a = torch.randn(nd * M, K, device=dev).to(torch.bfloat16)
        bt = torch.randn(nd, N, K, device=dev).to(torch.bfloat16)
        ops[name] = (a, bt[0] if nd == 1 else bt, M, N, K, nd)
        res = []
        for ns in (3, 4, 6):
            assert lib.skr_gemm_set_nstage(ns) == 0
            for bn in (64, 128):
                if ns == 6 and bn == 128:
                    continue
                for S in sorted({gemm.plan_splits(M, N, K, nd), 1, 2, 4, 8, 16, 32}):
                    if S < 1 or (K // 64) % S or N % bn:
                        continue
                    out = torch.empty(S, nd * M, N, device=dev)
                    us = timeit(lambda: gemm.rec_gemm(a, ops[name][1], out, S, nd, bn))
                    ref = (a.float().view(nd, M, K) @ bt.float().transpose(1, 2)).reshape(nd * M, N)
                    err = (out.sum(0) - ref).abs().max().item()
                    assert err < 1e-2 * ref.abs().max().item() + 1e-3, (name, S, err)
                    res.append("n%d/b%d/S%d %.1f" % (ns, bn, S, us))
        out1 = torch.empty(nd, M, N, device=dev)
        us_lib = timeit(lambda: torch.mm(a, bt[0].t(), out_dtype=torch.float32, out=out1[0]))
        print("%s M=%d N=%d K=%d  hipBLASLt %.1fus | plan S=%d | %s" % (
            name, M, N, K, us_lib, gemm.plan_splits(M, N, K, nd), " ".join(res)), flush=True)
    for gname, i, j in GROUPS:
        jobs = []
        for k in (i, j):
            a, bt, M, N, K, nd = ops[SHAPES[k][0]]
            S = gemm.plan_splits(M, N, K, nd)
            jobs.append((a, bt, torch.empty(S, M, N, device=dev), S))
        res = []
        for ns in (3, 4, 6):
            lib.skr_gemm_set_nstage(ns)
            res.append("n%d %.1f" % (ns, timeit(lambda: gemm.rec_gemm_group(jobs))))
        print("group %s: %s" % (gname, " ".join(res)), flush=True)
    lib.skr_gemm_set_nstage(3)


if __name__ == "__main__":
    main()
