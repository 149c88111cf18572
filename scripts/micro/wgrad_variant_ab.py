#!/usr/bin/env python3
"""Weight-gradient kernel schedules A/B (skr_wgrad_set_variant: 1 = 8 waves,
both k16 halves read up front; 2 = 4 waves of 128 x 128, fragments pipelined
across the K-step) on the vae_large step's shapes, alternating variants.
One JSON line per (shape, variant, round)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.ops import gemm  # noqa: E402
from sketch_rnn_amd.utils import native  # noqa: E402


def timeit(fn, reps=10):
    for _ in range(2):
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
    lib = native.require_hip().lib
    TB, bf = 25000, torch.bfloat16
    A2 = torch.randn(TB, 2304, device="cuda").to(bf)
    dRM = torch.randn(TB, 8192, device="cuda").to(bf)
    dRY = torch.randn(TB, 1024, device="cuda").to(bf)
    dVEC = torch.randn(TB, 24576, device="cuda").to(bf)
    Aenc = torch.randn(2, TB, 512, device="cuda").to(bf)
    dGenc = torch.randn(2, TB, 2048, device="cuda").to(bf)
    cases = [("dW_h", lambda: gemm.wgrad(A2[:, :2048], dRM), 2 * TB * 2048 * 8192),
             ("dP+cs", lambda: gemm.wgrad(A2[:, 2048:], dVEC, colsum=True), 2 * TB * 256 * 24576),
             ("dW_y", lambda: gemm.wgrad(A2, dRY), 2 * TB * 2304 * 1024),
             ("enc", lambda: gemm.wgrad(Aenc, dGenc), 2 * 2 * TB * 512 * 2048)]
    prev = lib.skr_wgrad_set_variant(-1)
    try:
        for rnd in range(2):
            for name, fn, fl in cases:
                for v in (1, 2):
                    lib.skr_wgrad_set_variant(v)
                    us = timeit(fn)
                    print(json.dumps({"shape": name, "variant": v, "round": rnd, "us": round(us, 1),
                                      "tflops": round(fl / us / 1e6, 1)}), flush=True)
    finally:
        lib.skr_wgrad_set_variant(prev)


if __name__ == "__main__":
    main()
