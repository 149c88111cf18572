#!/usr/bin/env python3
"""One weight-gradient shape of the vae_large step, repeated (for rocprofv3
--pmc passes over csrc/wgrad_gemm.hip): usage wgrad_one.py [dW_h|dP|dW_y|enc] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.ops import gemm  # noqa: E402


def main():
    shape = sys.argv[1] if len(sys.argv) > 1 else "dW_h"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    TB, bf = 25000, torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    A2 = torch.randn(TB, 2304, device="cuda", generator=g).to(bf)
    if shape == "dW_h":
        B = torch.randn(TB, 8192, device="cuda", generator=g).to(bf)
        fn = lambda: gemm.wgrad(A2[:, :2048], B)  # noqa: E731
    elif shape == "dP":
        B = torch.randn(TB, 24576, device="cuda", generator=g).to(bf)
        fn = lambda: gemm.wgrad(A2[:, 2048:], B, colsum=True)  # noqa: E731
    elif shape == "dW_y":
        B = torch.randn(TB, 1024, device="cuda", generator=g).to(bf)
        fn = lambda: gemm.wgrad(A2, B)  # noqa: E731
    else:
        A = torch.randn(2, TB, 512, device="cuda", generator=g).to(bf)
        B = torch.randn(2, TB, 2048, device="cuda", generator=g).to(bf)
        fn = lambda: gemm.wgrad(A, B)  # noqa: E731
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    print("done", shape, reps, flush=True)


if __name__ == "__main__":
    main()
