#!/usr/bin/env python3
"""Weight-gradient GEMM layouts of the vae_large step (K = T*B = 25000 rows):
times hipBLASLt on the layouts the backward can produce, to pick the fastest
formulation. usage: python scripts/bench_wgrad.py"""
import time

import torch


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
    dev, bf = "cuda", torch.bfloat16
    TB = 25000
    # dW_h: A2[:, :2048]^T @ dRM, A2 [TB, 2304] bf16, dRM [TB, 8192] bf16
    A2 = torch.randn(TB, 2304, device=dev).to(bf)
    dRM = torch.randn(TB, 8192, device=dev).to(bf)
    A2c = A2[:, :2048].contiguous()
    out = torch.empty(2048, 8192, device=dev)
    outT = torch.empty(8192, 2048, device=dev)
    fl = 2 * TB * 2048 * 8192
    def splitk(a, b, S):   # a [K, M], b [K, N] -> sum_s a_s^T b_s via one bmm
        K = a.shape[0]
        return torch.bmm(a.view(S, K // S, -1).transpose(1, 2), b.view(S, K // S, -1),
                         out_dtype=torch.float32).sum(0)

    for name, fn in [
        ("dW_h  splitK2", lambda: splitk(A2c, dRM, 2)),
        ("dW_h  splitK5", lambda: splitk(A2c, dRM, 5)),
        ("dW_h  A^T@B strided A", lambda: torch.mm(A2[:, :2048].t(), dRM, out_dtype=torch.float32, out=out)),
        ("dW_h  A^T@B contig A", lambda: torch.mm(A2c.t(), dRM, out_dtype=torch.float32, out=out)),
        ("dW_h^T B^T@A", lambda: torch.mm(dRM.t(), A2[:, :2048], out_dtype=torch.float32, out=outT)),
        ("dW_h  bf16 out", lambda: torch.mm(A2[:, :2048].t(), dRM)),
    ]:
        us = timeit(fn)
        print("%-26s %8.1f us  %6.1f TFLOP/s" % (name, us, fl / us / 1e6), flush=True)
    # encoder dW: 2 directions, [512 x TB/ ... ] (B=100 per direction)
    A = torch.randn(250, 200, 512, device=dev).to(bf)
    dG = torch.randn(250, 200, 2048, device=dev).to(bf)
    fl = 2 * 2 * 25000 * 512 * 2048

    def perm_bmm():
        An = A.view(250, 2, 100, 512).permute(1, 0, 2, 3).reshape(2, 25000, 512)
        dGn = dG.view(250, 2, 100, 2048).permute(1, 0, 2, 3).reshape(2, 25000, 2048)
        return torch.bmm(An.transpose(1, 2), dGn, out_dtype=torch.float32)

    An = A.view(250, 2, 100, 512).permute(1, 0, 2, 3).reshape(2, 25000, 512).contiguous()
    dGn = dG.view(250, 2, 100, 2048).permute(1, 0, 2, 3).reshape(2, 25000, 2048).contiguous()
    o1 = torch.empty(2, 512, 2048, device=dev)
    for name, fn in [
        ("enc dW permute+bmm", perm_bmm),
        ("enc dW bmm (contig)", lambda: torch.bmm(An.transpose(1, 2), dGn, out_dtype=torch.float32, out=o1)),
        ("enc dW 2x mm (contig)", lambda: [torch.mm(An[d].t(), dGn[d], out_dtype=torch.float32, out=o1[d])
                                            for d in range(2)]),
        ("enc dW bmm^T", lambda: torch.bmm(dGn.transpose(1, 2), An, out_dtype=torch.float32)),
        ("enc dW splitK5", lambda: torch.bmm(An.view(10, 5000, 512).transpose(1, 2), dGn.view(10, 5000, 2048),
                                             out_dtype=torch.float32).view(2, 5, 512, 2048).sum(1)),
        ("enc dW splitK10", lambda: torch.bmm(An.view(20, 2500, 512).transpose(1, 2), dGn.view(20, 2500, 2048),
                                              out_dtype=torch.float32).view(2, 10, 512, 2048).sum(1)),
        ("enc dW splitK25", lambda: torch.bmm(An.view(50, 1000, 512).transpose(1, 2), dGn.view(50, 1000, 2048),
                                              out_dtype=torch.float32).view(2, 25, 512, 2048).sum(1)),
    ]:
        us = timeit(fn)
        print("%-26s %8.1f us  %6.1f TFLOP/s" % (name, us, fl / us / 1e6), flush=True)
    # hyper-norm projections: dP = HH^T @ dVEC  [256 x TB] @ [TB x 24576]
    HH = torch.randn(TB, 264, device=dev).to(bf)
    dV = torch.randn(TB, 24576, device=dev).to(bf)
    fl = 2 * TB * 264 * 24576
    for name, fn in [
        ("dP HH1^T@dVEC (M=264)", lambda: torch.mm(HH.t(), dV, out_dtype=torch.float32)),
        ("dP^T dVEC^T@HH1", lambda: torch.mm(dV.t(), HH, out_dtype=torch.float32)),
        ("dP splitK5", lambda: splitk(HH, dV, 5)),
        ("dP splitK10", lambda: splitk(HH, dV, 10)),
    ]:
        us = timeit(fn)
        print("%-26s %8.1f us  %6.1f TFLOP/s" % (name, us, fl / us / 1e6), flush=True)


if __name__ == "__main__":
    main()
