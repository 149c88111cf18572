"""Column reductions for sequence parameter gradients (``csrc/reduce.hip``).

``colsum(x, y)`` returns ``(sum_rows(x * y), sum_rows(x))`` for ``x, y``
(fp32 or bf16, fp32 accumulation) shaped ``[R1, R2, C]`` (any strides with a contiguous last dim) -- the
LayerNorm gamma/beta and bias gradients of the recurrent layers, computed in
one pass over the saved ``[T*B, C]`` streams. PyTorch fallback on the CPU.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def colsum(x: torch.Tensor, y: Optional[torch.Tensor] = None, splits: Optional[int] = None
           ) -> Tuple[Optional[torch.Tensor], torch.Tensor]:
    """``splits``: row slices (workgroups per 256 columns); default fills
    ~1024 workgroups, so narrow outputs (a head bias: 123 columns) still
    spread over the chip."""
    if x.dim() == 2:
        x = x.unsqueeze(0)
        y = y.unsqueeze(0) if y is not None else None
    assert x.dim() == 3 and x.stride(-1) == 1
    from . import use_hip
    if not use_hip(x):
        xf = x.float()
        sxy = (xf * y.float()).sum((0, 1)) if y is not None else None
        return sxy, xf.sum((0, 1))
    from ..utils import native
    lib = native.require_hip()
    R1, R2, C = x.shape
    if y is not None:
        assert y.dtype in (torch.float32, torch.bfloat16) and y.shape == x.shape and y.stride() == x.stride()
    if splits is None:   # ~1024 workgroups; a thread sums 4 columns when C % 4 == 0 (csrc/reduce.hip)
        splits = -(-1024 // -(-C // (1024 if C % 4 == 0 else 256)))
    RS = max(1, min(splits, (R1 * R2) // 16))
    part = torch.empty(2, RS, C, device=x.device, dtype=torch.float32)
    tot = torch.empty(2, C, device=x.device, dtype=torch.float32)
    kind = 1 if x.dtype == torch.bfloat16 else 2
    assert x.dtype in (torch.bfloat16, torch.float32)
    ykind = 1 if (y is not None and y.dtype == torch.bfloat16) else 2
    # both passes in HIP: row-slice partials, then the fixed-order column totals
    rc = lib.lib.skr_colsum2(x.data_ptr(), kind, y.data_ptr() if y is not None else None, ykind, R1, x.stride(0), R2,
                             x.stride(1), C, RS, part[0].data_ptr(), part[1].data_ptr(), tot[0].data_ptr(),
                             tot[1].data_ptr(), torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_colsum failed (%d)" % rc)
    return (tot[0] if y is not None else None), tot[1]


# Columns per thread of colsum_many when every operand is bf16 (8: one
# 16-byte load per row and operand; 4: the A/B arm, 8-byte loads).
COLSUM_NC = 8


def colsum_many(pairs, splits=None):
    """:func:`colsum` of several ``(x, y)`` pairs (``[R, C]`` or ``[R1, R2, C]``
    views with a contiguous last dim, y may be None) in two launches for all of them (csrc/reduce.hip
    ``skr_colsum_multi``): the narrow reductions run beside the wide one
    instead of each paying a kernel boundary and a tail. ``splits``: a list
    of row-slice counts (default: :func:`colsum`'s, capped at 256 for
    C <= 1024 so their second pass stays short). C >= 1024: the same
    per-slice summation order as :func:`colsum` with the same splits;
    narrower reductions split each slice over row groups of one workgroup
    (summed in a fixed order). Falls back to one :func:`colsum` per pair
    off the vector path."""
    from . import use_hip
    pairs = [(x.unsqueeze(0), y.unsqueeze(0) if y is not None else None) if x.dim() == 2 else (x, y)
             for x, y in pairs]
    if not pairs or len(pairs) > 4 or not all(
            use_hip(x) and x.dim() == 3 and x.stride(-1) == 1 and x.shape[-1] % 4 == 0 and x.stride(0) % 4 == 0
            and (x.shape[-1] >= 1024 or 256 % (x.shape[-1] // 4) == 0)
            and x.stride(1) % 4 == 0
            and x.dtype in (torch.bfloat16, torch.float32) and x.data_ptr() % 16 == 0
            and (y is None or (y.shape == x.shape and y.stride() == x.stride() and y.data_ptr() % 16 == 0
                               and y.dtype in (torch.bfloat16, torch.float32)))
            for x, y in pairs):
        return [colsum(x, y, splits[i] if splits else None) for i, (x, y) in enumerate(pairs)]
    from ..utils import native
    from ._hipapi import CsJob
    lib = native.require_hip()
    jobs = (CsJob * len(pairs))()
    keep, outs = [], []
    # 8 columns per thread: bf16 operands, C and the row strides multiples of 8
    # (narrow C: C / 8 divides 256); the row slices are sized for the
    # workgroup's 256 * nc columns
    nc = 8 if COLSUM_NC == 8 and all(
        x.dtype == torch.bfloat16 and (y is None or y.dtype == torch.bfloat16) and x.shape[-1] % 8 == 0
        and x.stride(0) % 8 == 0 and x.stride(1) % 8 == 0 and (x.shape[-1] >= 2048 or 256 % (x.shape[-1] // 8) == 0)
        for x, y in pairs) else 4
    # the widest (longest-running) reduction's workgroups are dispatched
    # first; the narrow ones fill the slots beside and after it
    order = sorted(range(len(pairs)), key=lambda i: -pairs[i][0].shape[-1])
    for slot, i in enumerate(order):
        x, y = pairs[i]
        R1, R2, C = x.shape
        R = R1 * R2
        if splits:
            RS = splits[i]
        else:
            RS = -(-1024 // -(-C // (256 * nc)))
            if C <= 256 * nc:
                RS = min(RS, 256)
        RS = max(1, min(RS, R // 16))
        part = torch.empty(2, RS, C, device=x.device, dtype=torch.float32)
        tot = torch.empty(2, C, device=x.device, dtype=torch.float32)
        J = jobs[slot]
        J.X, J.Y = x.data_ptr(), (y.data_ptr() if y is not None else None)
        J.R1, J.s1, J.R2, J.s2 = R1, x.stride(0), R2, x.stride(1)
        J.C, J.RS = C, RS
        J.xbf, J.ybf = int(x.dtype == torch.bfloat16), int(y is not None and y.dtype == torch.bfloat16)
        J.part_xy, J.part_x = part[0].data_ptr(), part[1].data_ptr()
        J.out_xy, J.out_x = tot[0].data_ptr(), tot[1].data_ptr()
        keep.append(part)
        outs.append((i, tot, y is not None))
    rc = lib.lib.skr_colsum_multi(jobs, len(pairs), nc, torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_colsum_multi failed (%d)" % rc)
    res = [None] * len(pairs)
    for i, tot, hy in outs:
        res[i] = ((tot[0] if hy else None), tot[1])
    return res
