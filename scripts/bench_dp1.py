#!/usr/bin/env python3
"""Microbenchmark: the HyperLSTM hyper-norm projection gradient
dP1 = [hh | 1]^T @ dvec over T*B = 25000 rows (vae_large: hh 256 wide, dvec
12*2048 wide, bf16 operands, fp32 output) in several formulations."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from sketch_rnn_amd.ops import gemm  # noqa: E402
from sketch_rnn_amd.ops.reduce import colsum  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    TB, Hh, N = 25000, 256, 12 * 2048
    dev, bf = "cuda", torch.bfloat16
    hh = torch.randn(TB, Hh, device=dev).to(bf)
    dv = (torch.randn(TB, N, device=dev) * 0.01).to(bf)
    res = {}
    for pad in (8, 16, 64):
        h1 = torch.zeros(TB, Hh + pad, device=dev, dtype=bf)
        h1[:, :Hh] = hh
        h1[:, Hh] = 1.0
        res["ones_row_M%d" % (Hh + pad)] = timeit(lambda: gemm.wgrad(h1, dv))
        res["ones_row_T_N%d" % (Hh + pad)] = timeit(lambda: gemm.wgrad(dv, h1))
    res["M256_plus_colsum"] = timeit(lambda: (gemm.wgrad(hh, dv), colsum(dv)))
    res["M256_only"] = timeit(lambda: gemm.wgrad(hh, dv))
    res["colsum_only"] = timeit(lambda: colsum(dv))
    for k, v in res.items():
        print("%-22s %8.1f us" % (k, v), flush=True)


if __name__ == "__main__":
    main()
