#!/usr/bin/env python3
"""Diagnose the MX-fp8 GEMM's scale handling: one 128 x 128 x K product per
case with controlled operands (small-integer e4m3 values, exact in fp32),
reporting the max error relative to the output magnitude.

cases: unity scales; A scale by row; A scale by 32-k block index (0..3 within
a K-step); A scale by K-step; the same for W; both random."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd.ops import mx8  # noqa: E402


def blocks_to_scales(Sb):
    """[R, K/32] block-order scale bytes -> the kernels' [R][4][K/128] layout."""
    R, nb = Sb.shape
    return Sb.view(R, nb // 4, 4).transpose(1, 2).reshape(R, nb).contiguous()


def run(name, M, N, K, sa_fn, sw_fn, g):
    a = torch.randint(-3, 4, (M, K), device="cuda", generator=g).float()
    w = torch.randint(-3, 4, (N, K), device="cuda", generator=g).float()
    A8 = a.to(torch.float8_e4m3fn).view(torch.uint8)
    W8 = w.to(torch.float8_e4m3fn).view(torch.uint8)
    r = torch.arange(M, device="cuda").view(M, 1).expand(M, K // 32)
    c = torch.arange(N, device="cuda").view(N, 1).expand(N, K // 32)
    ba = torch.arange(K // 32, device="cuda").view(1, -1).expand(M, K // 32)
    bw = torch.arange(K // 32, device="cuda").view(1, -1).expand(N, K // 32)
    ea = sa_fn(r, ba)          # exponent offsets per (row, block), small ints
    ew = sw_fn(c, bw)
    SA = blocks_to_scales((127 + ea).to(torch.uint8))
    SW = blocks_to_scales((127 + ew).to(torch.uint8))
    C = mx8.gemm(A8.contiguous(), SA, W8.contiguous(), SW)
    ad = (a.view(M, K // 32, 32) * torch.exp2(ea.float()).unsqueeze(-1)).view(M, K).double()
    wd = (w.view(N, K // 32, 32) * torch.exp2(ew.float()).unsqueeze(-1)).view(N, K).double()
    ref = ad @ wd.t()
    mag = ad.abs() @ wd.abs().t()
    err = ((C.double() - ref).abs() / mag.clamp_min(1e-30)).max().item()
    # which (block) hypothesis fits: try the K-step-major reading of the scales
    print(json.dumps({"case": name, "M": M, "N": N, "K": K, "max_rel_err": round(err, 6),
                      "exact": bool(err < 1e-6)}), flush=True)


def mapping():
    """Which lane group's scale the hardware applies to each k of a K-step:
    row r of A has a single 1 at k = r (r < 128), its block scales are
    2^(j + 1) for lane group / block j, W is all ones with unit scales, so
    C[r, 0] = 2^(j(r) + 1)."""
    M = N = 128
    K = 512
    a = torch.zeros(M, K, device="cuda")
    a[torch.arange(128), torch.arange(128)] = 1.0
    A8 = a.to(torch.float8_e4m3fn).view(torch.uint8).contiguous()
    W8 = torch.ones(N, K, device="cuda").to(torch.float8_e4m3fn).view(torch.uint8).contiguous()
    Sb = torch.full((M, K // 32), 127, dtype=torch.uint8, device="cuda")
    Sb[:, 0:4] = torch.tensor([128, 129, 130, 131], dtype=torch.uint8, device="cuda")
    SW = torch.full((N, K // 32), 127, dtype=torch.uint8, device="cuda")
    C = mx8.gemm(A8, blocks_to_scales(Sb), W8, SW)
    j = torch.log2(C[:, 0]).round().long() - 1
    print(json.dumps({"case": "scale_group_of_k", "groups": j.tolist()}), flush=True)


def main():
    from sketch_rnn_amd.utils import native
    lib = native.require_hip().lib
    for layout in (0, 1):
        lib.skr_mx8_set_layout(layout)
        print(json.dumps({"layout": layout}), flush=True)
        mapping()
        _cases()
    lib.skr_mx8_set_layout(1)


def _cases():
    g = torch.Generator(device="cuda").manual_seed(0)
    zero = lambda r, b: torch.zeros_like(r)  # noqa: E731
    for K in (512,):
        M = N = 128
        run("unity", M, N, K, zero, zero, g)
        run("A_by_row", M, N, K, lambda r, b: (r % 5) - 2, zero, g)
        run("A_by_block_in_step", M, N, K, lambda r, b: (b % 4) - 1, zero, g)
        run("A_by_kstep", M, N, K, lambda r, b: (b // 4) % 3 - 1, zero, g)
        run("W_by_col", M, N, K, zero, lambda c, b: (c % 5) - 2, g)
        run("W_by_block_in_step", M, N, K, zero, lambda c, b: (b % 4) - 1, g)
        run("W_by_kstep", M, N, K, zero, lambda c, b: (b // 4) % 3 - 1, g)
        run("A_row_and_block", M, N, K, lambda r, b: ((r * 7 + b * 3) % 5) - 2, zero, g)
        run("both", M, N, K, lambda r, b: ((r * 7 + b * 3) % 5) - 2, lambda c, b: ((c * 5 + b) % 5) - 2, g)


if __name__ == "__main__":
    main()
