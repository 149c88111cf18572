"""MX-fp8 operands and GEMM (``csrc/mx8_gemm.hip``): OCP e4m3 values with
one E8M0 scale per 32 consecutive k of a row, the block format gfx950's
``v_mfma_scale_f32_16x16x128_f8f6f4`` consumes at twice the bf16 MFMA rate.
Used by the fp8 decode step (BASELINE config 5, ``sample/hyper_step.py``):
the weight is quantized once per weight version, the activation rows by the
cell that produces them.

Scale layout ``[rows][4][K/128]``: block ``b = k // 32`` of row ``r`` at
``r * K/32 + (b % 4) * K/128 + b // 4`` (:func:`scales_to_blocks` converts to
the natural ``[rows][K/32]`` order)."""
from __future__ import annotations

from typing import Tuple

import torch

from ..utils import native


def _lib():
    return native.require_hip().lib


def _st():
    return torch.cuda.current_stream().cuda_stream


def quant_t(W: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """fp32 weight ``W [K, N]`` -> ``(Q [N, K] uint8 e4m3, S [N, K/32] uint8 E8M0)``."""
    assert W.dtype == torch.float32 and W.stride(1) == 1 and W.is_cuda
    K, N = W.shape
    Q = torch.empty(N, K, dtype=torch.uint8, device=W.device)
    S = torch.empty(N, K // 32, dtype=torch.uint8, device=W.device)
    rc = _lib().skr_mx8_quant_t(W.data_ptr(), W.stride(0), K, N, Q.data_ptr(), S.data_ptr(), _st())
    if rc != 0:
        raise RuntimeError("skr_mx8_quant_t failed (%d) for [%d, %d]" % (rc, K, N))
    return Q, S


def quant_rows(A: torch.Tensor, Q: torch.Tensor = None, S: torch.Tensor = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rows of ``A [M, K]`` (bf16 or fp32) -> ``(Q [M, K], S [M, K/32])``."""
    assert A.dtype in (torch.bfloat16, torch.float32) and A.stride(1) == 1 and A.is_cuda
    M, K = A.shape
    Q = torch.empty(M, K, dtype=torch.uint8, device=A.device) if Q is None else Q
    S = torch.empty(M, K // 32, dtype=torch.uint8, device=A.device) if S is None else S
    rc = _lib().skr_mx8_quant_rows(A.data_ptr(), A.stride(0), int(A.dtype == torch.bfloat16), M, K, Q.data_ptr(),
                                   Q.stride(0), S.data_ptr(), _st())
    if rc != 0:
        raise RuntimeError("skr_mx8_quant_rows failed (%d) for [%d, %d]" % (rc, M, K))
    return Q, S


def gemm(A8: torch.Tensor, SA: torch.Tensor, W8: torch.Tensor, SW: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """``C [M, N] = (A8, SA) . (W8, SW)^T`` in fp32 (N % 128 == 0, K % 512 == 0, K <= 2048)."""
    M, K = A8.shape
    N = W8.shape[0]
    C = torch.empty(M, N, dtype=torch.float32, device=A8.device) if out is None else out
    assert C.stride(1) == 1 and tuple(C.shape) == (M, N)
    rc = _lib().skr_mx8_gemm(A8.data_ptr(), A8.stride(0), SA.data_ptr(), W8.data_ptr(), W8.stride(0), SW.data_ptr(),
                             C.data_ptr(), C.stride(0), M, N, K, _st())
    if rc != 0:
        raise RuntimeError("skr_mx8_gemm failed (%d) for M=%d N=%d K=%d" % (rc, M, N, K))
    return C


def scales_to_blocks(S: torch.Tensor) -> torch.Tensor:
    """``[rows][4][K/128]`` scale bytes -> ``[rows][K/32]`` in block order."""
    R, nb = S.shape
    return S.view(R, 4, nb // 4).transpose(1, 2).reshape(R, nb)


def dequant(Q: torch.Tensor, S: torch.Tensor) -> torch.Tensor:
    """fp32 values of an MX-fp8 tensor (torch's OCP ``float8_e4m3fn`` decode)."""
    R, K = Q.shape
    v = Q.view(torch.float8_e4m3fn).float().view(R, K // 32, 32)
    sc = torch.exp2(scales_to_blocks(S).float() - 127.0).unsqueeze(-1)
    return (v * sc).view(R, K)


def quant_ref(X: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """PyTorch transcription of the kernels' quantizer (rows of ``X [R, K]``,
    fp32): E8M0 exponent = biased exponent of the block amax - 7 (clamped to
    [0, 254]), values / 2^(X - 127) rounded to e4m3 (round to nearest even)."""
    R, K = X.shape
    blk = X.float().view(R, K // 32, 32)
    amax = blk.abs().amax(-1)
    e = ((amax.view(torch.int32) >> 23) & 0xff).long()
    Xe = (e - 7).clamp(0, 254)
    q = (blk * torch.exp2(127.0 - Xe.float()).unsqueeze(-1)).to(torch.float8_e4m3fn).view(torch.uint8).view(R, K)
    S = Xe.to(torch.uint8)                                   # [R, K/32] block order
    S = S.view(R, K // 128, 4).transpose(1, 2).reshape(R, K // 32)
    return q, S
