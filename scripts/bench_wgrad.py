#!/usr/bin/env python3
"""Weight-gradient GEMMs of the vae_large step (K = T*B = 25000 rows): the
hand-written kernel (csrc/wgrad_gemm.hip) against the hipBLASLt formulation
(``SKR_WGRAD_HIP=0`` path of ops.gemm.wgrad) on every shape the backward
issues. One JSON line per shape. usage: python scripts/bench_wgrad.py"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.ops import gemm  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    dev, bf = "cuda", torch.bfloat16
    TB = 25000
    A2 = torch.randn(TB, 2304, device=dev).to(bf)          # decoder [h | hh] rows
    dRM = torch.randn(TB, 8192, device=dev).to(bf)
    dRY = torch.randn(TB, 1024, device=dev).to(bf)
    dVEC = torch.randn(TB, 24576, device=dev).to(bf)
    Aenc = torch.randn(2, TB, 512, device=dev).to(bf)       # encoder directions
    dGenc = torch.randn(2, TB, 2048, device=dev).to(bf)
    cases = [
        ("dW_h [2048 x 8192]", lambda: gemm.wgrad(A2[:, :2048], dRM), 2 * TB * 2048 * 8192),
        ("dP + colsum [256 x 24576]", lambda: gemm.wgrad(A2[:, 2048:], dVEC, colsum=True), 2 * TB * 256 * 24576),
        ("dW_y [2304 x 1024]", lambda: gemm.wgrad(A2, dRY), 2 * TB * 2304 * 1024),
        ("enc dW 2 x [512 x 2048]", lambda: gemm.wgrad(Aenc, dGenc), 2 * 2 * TB * 512 * 2048),
    ]
    if "--sweep" in sys.argv:   # split-K counts x fragment schedules of the hand-written kernel
        lib = __import__("sketch_rnn_amd.utils.native", fromlist=["x"]).require_hip().lib
        shapes = {"dW_h": (2048, 8192, 1), "dP": (256, 24576, 1), "dW_y": (2304, 1024, 1), "enc": (512, 2048, 2)}
        for (name, fn, fl), key in zip(cases, shapes):
            for db in (0, 1):
                lib.skr_wgrad_set_variant(db)
                for S in (1, 2, 3, 4, 5, 6, 7, 8, 9, 10):
                    M, N, nb = shapes[key]
                    tiles = nb * (M // 256) * (N // 256)
                    if tiles * S > 1024 or (S > 1 and tiles >= 192 and S > 2):
                        continue
                    gemm.WGRAD_SPLIT = {shapes[key]: S}
                    us = timeit(fn)
                    print(json.dumps({"shape": key, "db": db, "S": S, "us": round(us, 1),
                                      "tflops": round(fl / us / 1e6, 1)}), flush=True)
        gemm.WGRAD_SPLIT = {}
        lib.skr_wgrad_set_variant(0)
        return
    impls = ("hip", "hipblaslt")
    tot = {k: 0.0 for k in impls}
    for name, fn, fl in cases:
        rec = {"shape": name}
        for impl in impls:
            gemm.WGRAD_HIP = impl != "hipblaslt"
            us = timeit(fn)
            tot[impl] += us
            rec[impl + "_us"] = round(us, 1)
            rec[impl + "_tflops"] = round(fl / us / 1e6, 1)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us": {k: round(v, 1) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
