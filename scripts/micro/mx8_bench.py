#!/usr/bin/env python3
"""h W_h of the decode step at B rows (vae_large: K = H = 2048, N = 4H =
8192): the MX-fp8 GEMM (csrc/mx8_gemm.hip) against the bf16 skinny GEMM the
step uses today (ops.gemm.rec_gemm: 128-row blocks, split-K slabs). Device
time per call from graph-replayed batches of 20 calls. One JSON line per B."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.ops import gemm, mx8  # noqa: E402


def per_call_us(fn, n=20, reps=5):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return 1000 * e0.elapsed_time(e1) / reps / n


def main():
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    K, N = 2048, 8192
    W = torch.randn(K, N, device="cuda") * 0.02
    WT = W.t().contiguous().to(torch.bfloat16)
    W8, SW = mx8.quant_t(W)
    for B in (128, 256, 512, 1024):
        h = torch.tanh(torch.randn(B, K, device="cuda"))
        hb = h.to(torch.bfloat16)
        A8, SA = mx8.quant_rows(h)
        S = 4 if B <= 128 else 1
        R = torch.empty(S, B, N, device="cuda")
        C = torch.empty(B, N, device="cuda")
        t_bf = per_call_us(lambda: gemm.rec_gemm(hb, WT, R, S))
        t_f8 = per_call_us(lambda: mx8.gemm(A8, SA, W8, SW, out=C))
        ref = h.double() @ W.double()
        err = float((C.double() - ref).norm() / ref.norm())
        print(json.dumps({"B": B, "N": N, "K": K, "bf16_skinny_us": round(t_bf, 2), "mx8_us": round(t_f8, 2),
                          "speedup": round(t_bf / t_f8, 2), "mx8_rel_err_vs_fp64": round(err, 5),
                          "mx8_tflops": round(2 * B * N * K / t_f8 / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
