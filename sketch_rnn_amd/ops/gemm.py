"""GEMM dispatch with a selectable operand precision (fp32 / bf16).

Where each product runs (vae_large: no library GEMM in the profile,
profiles/r3/vae_large_kernel_summary.txt):

* per-time-step recurrent products (``h @ W_h``, the grouped HyperLSTM
  products, their backward twins): hand-written MFMA skinny split-K GEMMs,
  ``csrc/skinny_gemm.hip`` (:func:`rec_gemm`, :func:`rec_gemm_group`);
* long-K weight gradients over all T*B rows: ``csrc/wgrad_gemm.hip``
  (:func:`wgrad`; bf16, 256-multiple shapes);
* small products (z-projections, hyper-norm factors): ``csrc/small_gemm.hip``
  (:func:`small_mm`, :func:`small_mm_batched`);
* everything else -- fp32 / odd-shaped weight gradients (:func:`wgrad`'s
  fallback), the generic :func:`mm` / :func:`bmm` helpers used off the
  flagship path -- goes to hipBLASLt through torch. In ``bf16`` mode
  operands are bf16 and results fp32 (``torch.mm(..., out_dtype=float32)``),
  so accumulation and everything downstream stay fp32.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import get_compute_dtype

_BF16 = torch.bfloat16


def lp_dtype() -> torch.dtype:
    return _BF16 if get_compute_dtype() == "bf16" else torch.float32


def lp(t: torch.Tensor) -> torch.Tensor:
    d = lp_dtype()
    return t if t.dtype == d else t.to(d)


def mm(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``a @ b`` with fp32 output; operands used as given (fp32 or bf16)."""
    if a.dtype == torch.float32 and b.dtype == torch.float32:
        return torch.mm(a, b, out=out) if out is not None else torch.mm(a, b)
    if a.dtype != b.dtype:
        a, b = a.to(_BF16), b.to(_BF16)
    if out is not None:
        return torch.mm(a, b, out_dtype=torch.float32, out=out)
    return torch.mm(a, b, out_dtype=torch.float32)


_ONES = {}


def ones_row(n: int, device) -> torch.Tensor:
    """``[1, n]`` fp32 ones: the A operand that turns a :class:`SmallGroup`
    product into a column sum (``ones @ P`` = ``P.sum(0)``) inside the same
    grouped launch. Cached per (device, n) when created eagerly; a tensor
    first asked for during HIP-graph capture is not cached (it lives in the
    graph's pool)."""
    dev = torch.device(device)
    key = (dev, int(n))
    t = _ONES.get(key)
    if t is None:
        t = torch.ones(1, n, device=dev)
        if not (dev.type == "cuda" and torch.cuda.is_current_stream_capturing()):
            _ONES[key] = t
    return t


def small_mm(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None, acc: bool = False) -> torch.Tensor:
    """fp32 ``a @ b (+ bias) (+ out if acc)`` for the small per-sequence
    products (latent heads, initial state, z projections and their grads):
    ``csrc/small_gemm.hip`` on the GPU -- operands may be transposed views
    (arbitrary strides, no copies), deterministic split-K -- and torch
    elsewhere. ``out`` needs unit column stride."""
    M, K = a.shape
    N = b.shape[1]
    if not a.is_cuda:
        y = a @ b
        if bias is not None:
            y = y + bias
        if out is None:
            return y
        if acc:
            out += y
        else:
            out.copy_(y)
        return out
    from ..utils import native
    lib = native.require_hip().lib
    assert a.dtype == b.dtype == torch.float32 and b.shape[0] == K
    if out is None:
        out = torch.empty(M, N, device=a.device)
    assert out.stride(1) == 1 and out.shape == (M, N)
    S = lib.skr_small_gemm_splits(M, N, K)
    work = torch.empty(S * M * N if S > 1 else 1, device=a.device)
    bc = bias.contiguous() if bias is not None else None
    rc = lib.skr_small_gemm(a.data_ptr(), a.stride(0), a.stride(1), b.data_ptr(), b.stride(0), b.stride(1),
                            out.data_ptr(), out.stride(0), bc.data_ptr() if bc is not None else None, M, N, K,
                            int(acc), work.data_ptr(), work.numel(), torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_small_gemm failed (%d) for M=%d N=%d K=%d" % (rc, M, N, K))
    return out


def small_mm_batched(a: torch.Tensor, a_off: int, a_batch: int, sam: int, sak: int,
                     b: torch.Tensor, b_off: int, b_batch: int, sbk: int, sbn: int,
                     c: torch.Tensor, c_off: int, c_batch: int, ldc: int,
                     M: int, N: int, K: int, nbatch: int, acc: bool = False) -> None:
    """``nbatch`` fp32 products on raw element strides (``csrc/small_gemm.hip``):
    for batch i, ``C_i[m, n] (+)= sum_k A_i[m*sam + k*sak] B_i[k*sbk + n*sbn]``
    with ``A_i = a + a_off + i*a_batch`` (likewise B, C). Used where the
    operands are blocks of one buffer that no single view describes (the
    per-block hyper-projection gradients)."""
    from ..utils import native
    lib = native.require_hip().lib
    assert a.dtype == b.dtype == c.dtype == torch.float32
    S = lib.skr_small_gemm_splits(M, N, K)
    work = torch.empty(nbatch * S * M * N if S > 1 else 1, device=c.device)
    rc = lib.skr_small_gemm_batched(a.data_ptr() + 4 * a_off, a_batch, sam, sak, b.data_ptr() + 4 * b_off, b_batch,
                                    sbk, sbn, c.data_ptr() + 4 * c_off, c_batch, ldc, None, M, N, K, int(acc), nbatch,
                                    work.data_ptr(), work.numel(), torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_small_gemm_batched failed (%d) for M=%d N=%d K=%d x%d" % (rc, M, N, K, nbatch))


class SmallGroup:
    """Independent :func:`small_mm` / :func:`small_mm_batched` products
    collected and run as ONE grouped launch (+ one split-K sum launch;
    ``csrc/small_gemm.hip`` ``skr_small_gemm_group``): the same tiles and
    summation order as the single calls, so the results are identical. On
    the CPU each product runs immediately. Usage::

        g = SmallGroup(device)
        mu = g.mm(h, w_mu, b_mu)
        ps = g.mm(h, w_sig, b_sig)
        g.run()            # mu, ps are valid after this
    """

    MAX = 6

    def __init__(self, device):
        self.dev = torch.device(device)
        self.items = []

    def mm(self, a, b, bias=None, out=None, acc=False):
        if not a.is_cuda:
            return small_mm(a, b, bias, out, acc)
        M, K = a.shape
        N = b.shape[1]
        assert a.dtype == b.dtype == torch.float32 and b.shape[0] == K
        if out is None:
            out = torch.empty(M, N, device=a.device)
        assert out.stride(1) == 1 and out.shape == (M, N)
        bc = bias.contiguous() if bias is not None else None
        self.items.append(dict(A=a, a_off=0, sam=a.stride(0), sak=a.stride(1), a_batch=0, B=b, b_off=0,
                               sbk=b.stride(0), sbn=b.stride(1), b_batch=0, C=out, c_off=0, ldc=out.stride(0),
                               c_batch=0, bias=bc, M=M, N=N, K=K, acc=int(acc), nbatch=1))
        return out

    def batched(self, a, a_off, a_batch, sam, sak, b, b_off, b_batch, sbk, sbn, c, c_off, c_batch, ldc, M, N, K,
                nbatch, acc=False):
        assert a.is_cuda and a.dtype == b.dtype == c.dtype == torch.float32
        self.items.append(dict(A=a, a_off=a_off, sam=sam, sak=sak, a_batch=a_batch, B=b, b_off=b_off, sbk=sbk,
                               sbn=sbn, b_batch=b_batch, C=c, c_off=c_off, ldc=ldc, c_batch=c_batch, bias=None,
                               M=M, N=N, K=K, acc=int(acc), nbatch=nbatch))

    def run(self) -> None:
        if not self.items:
            return
        from ..utils import native
        from ._hipapi import SgProb
        lib = native.require_hip().lib
        for i0 in range(0, len(self.items), self.MAX):
            chunk = self.items[i0:i0 + self.MAX]
            probs = (SgProb * len(chunk))()
            keep = []
            for p, it in zip(probs, chunk):
                S = lib.skr_small_gemm_splits(it["M"], it["N"], it["K"])
                work = torch.empty(it["nbatch"] * S * it["M"] * it["N"] if S > 1 else 1, device=self.dev)
                keep.append(work)
                p.A, p.sam, p.sak, p.a_batch = it["A"].data_ptr() + 4 * it["a_off"], it["sam"], it["sak"], it["a_batch"]
                p.B, p.sbk, p.sbn, p.b_batch = it["B"].data_ptr() + 4 * it["b_off"], it["sbk"], it["sbn"], it["b_batch"]
                p.C, p.ldc, p.c_batch = it["C"].data_ptr() + 4 * it["c_off"], it["ldc"], it["c_batch"]
                p.bias = it["bias"].data_ptr() if it["bias"] is not None else None
                p.M, p.N, p.K, p.acc, p.nbatch = it["M"], it["N"], it["K"], it["acc"], it["nbatch"]
                p.work, p.work_elems = work.data_ptr(), work.numel()
            rc = lib.skr_small_gemm_group(probs, len(chunk), torch.cuda.current_stream().cuda_stream)
            if rc != 0:
                raise RuntimeError("skr_small_gemm_group failed (%d)" % rc)
        self.items = []


def bmm(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if a.dtype == torch.float32 and b.dtype == torch.float32:
        return torch.bmm(a, b, out=out) if out is not None else torch.bmm(a, b)
    if out is not None:
        return torch.bmm(a, b, out_dtype=torch.float32, out=out)
    return torch.bmm(a, b, out_dtype=torch.float32)


def _wgrad_hip_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Shapes the hand-written kernel (csrc/wgrad_gemm.hip) takes: bf16
    operands on the GPU, M and N multiples of its 256 x 256 output tile,
    rows 16-byte aligned (anything else: hipBLASLt)."""
    from . import use_hip
    if not (WGRAD_HIP and a.is_cuda and use_hip(a) and a.dtype == _BF16 and b.dtype == _BF16):
        return False
    M, N = a.shape[-1], b.shape[-1]
    return (M % 256 == 0 and N % 256 == 0 and a.stride(-1) == 1 and b.stride(-1) == 1
            and all(st % 8 == 0 for st in a.stride()[:-1] + b.stride()[:-1])
            and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0)


WGRAD_HIP = True   # False: hipBLASLt weight gradients (tests / A-B)
WGRAD_SPLIT = {}   # (M, N, batch) -> split-K count override (scripts/bench_wgrad.py sweeps)
# Weight-gradient kernel schedule (csrc/wgrad_gemm.hip skr_wgrad_set_variant):
# 1 = 8 waves of 64 x 128, both k16 halves' fragments read up front; 2 = 4
# waves of 128 x 128, fragments pipelined across the K-step (bit-identical
# products; measured slower on every step shape, profiles/r6/wgrad_variant_ab.jsonl).
# None leaves the library's setting.
WGRAD_KERNEL = None


def grad_slot(param: torch.Tensor, shape) -> Optional[torch.Tensor]:
    """The optimizer-arena slice reserved for ``param``'s gradient
    (train/optim.py FlatAdam) when it has exactly ``shape`` and is
    contiguous: a weight-gradient kernel writes there directly, and the
    tensor it returns becomes ``param.grad`` without a copy."""
    t = getattr(param, "_grad_slot", None)
    # only while the gradient is unbound (zero_grad(set_to_none=True)): with
    # param.grad set to the slot, autograd would add the slot to itself
    if t is None or param.grad is not None or tuple(t.shape) != tuple(shape) or not t.is_contiguous() or t.dtype != torch.float32:
        return None
    # a FRESH view: autograd's AccumulateGrad adopts a gradient tensor only
    # when nothing else references it -- the slot tensor itself (held by
    # param._grad_slot) would be cloned, and gather_grads would copy it back
    return t.view(t.shape)


def grad_span(first: torch.Tensor, last: torch.Tensor, start: int, shape) -> Optional[torch.Tensor]:
    """A fresh view of the optimizer arena covering ``numel(shape)`` floats
    from element ``start`` of ``first``'s gradient slot -- reaching into the
    slots of the parameters that follow it, up to ``last`` -- when those
    slots are consecutive in the arena and every gradient is unbound (else
    None). One kernel then writes a product whose rows are split over several
    parameters (the HyperLSTM's [W_y_h; W_y_hh] weight gradient) in place."""
    a, b = getattr(first, "_grad_slot", None), getattr(last, "_grad_slot", None)
    if a is None or b is None or first.grad is not None or last.grad is not None:
        return None
    n = 1
    for d in shape:
        n *= d
    end = b.data_ptr() + b.numel() * 4
    if a.dtype != torch.float32 or a.data_ptr() + (start + n) * 4 != end:
        return None
    base = a.view(-1)
    full = torch.as_strided(base, (n,), (1,), base.storage_offset() + start)
    return full.view(*shape)


def _wgrad_splits(tiles: int, K: int) -> int:
    """Split-K count of the long-K weight-gradient kernel. One workgroup per
    CU holds a 256 x 256 tile, so the run takes ceil(tiles * S / 256) rounds
    of K / (32 S) K-steps (~1 us each), plus the fp32 partial slabs written
    and summed (~0.1 us per slab tile). Measured (profiles/r5/wgrad_sweep.jsonl):
    dP 96 tiles S = 5 (438 us) against the old whole-wave rule's S = 2 (514);
    dW_y 36 tiles S = 7; encoder 32 tiles S = 8; dW_h 256 tiles S = 1; the
    MDN head's [Hd x 256] gradient (8 tiles) S = 32."""
    best, pick = None, 1
    for S in range(1, 33):
        if S > 1 and K // S < 512:   # at least 512 rows per split
            break
        cost = -(-tiles * S // 256) * (K / 32.0 / S) + 0.1 * tiles * S
        if best is None or cost < best - 1e-9:
            best, pick = cost, S
    return pick


def _wgrad_hip(a, b, colsum, out=None, acc=False, max_grid=0, cs=None):
    from ..utils import native
    lib = native.require_hip()
    if WGRAD_KERNEL is not None:
        lib.lib.skr_wgrad_set_variant(int(WGRAD_KERNEL))
    n, K, M = a.shape
    N = b.shape[-1]
    tiles = n * (M // 256) * (N // 256)
    # a bounded grid walks the tiles itself: no split-K (the launch is meant
    # to leave most CUs to the stream it runs beside)
    S = 1 if max_grid > 0 else WGRAD_SPLIT.get((M, N, n), _wgrad_splits(tiles, K))
    dev = a.device
    out = out.view(n, M, N) if out is not None else torch.empty(n, M, N, device=dev, dtype=torch.float32)
    work = torch.empty(n * S, M, N, device=dev, dtype=torch.float32) if S > 1 else None
    if colsum:
        cs = cs.view(n, N) if cs is not None else torch.empty(n, N, device=dev, dtype=torch.float32)
    else:
        cs = None
    csw = torch.empty(n * S, N, device=dev, dtype=torch.float32) if (colsum and S > 1) else None
    ptr = lambda t: t.data_ptr() if t is not None else None
    rc = lib.lib.skr_wgrad2(a.data_ptr(), a.stride(1), a.stride(0) if n > 1 else 0, b.data_ptr(), b.stride(1),
                            b.stride(0) if n > 1 else 0, K, M, N, n, S, out.data_ptr(), ptr(work), ptr(cs), ptr(csw),
                            int(acc), int(max_grid), torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_wgrad failed (%d) for [%d, %d]^T [%d, %d] x %d" % (rc, K, M, K, N, n))
    return out, cs


class Background:
    """Kernels issued on a per-device side stream behind everything the
    current stream has queued so far (an event wait), joined back with
    :meth:`join`. Inside a graph capture the side stream joins the capture
    through that wait, so the captured graph holds the side work as a
    parallel branch. Used for the HyperLSTM weight gradients that run beside
    the backward scan (ops/hyper.py): callers allocate every tensor the side
    work writes on the current stream first and join before those tensors
    (or the inputs the side work reads) are used or freed."""

    _streams = {}

    def __init__(self, device):
        device = torch.device(device)
        self.main = torch.cuda.current_stream(device)
        key = device.index if device.index is not None else torch.cuda.current_device()
        if key not in Background._streams:
            Background._streams[key] = torch.cuda.Stream(device)
        self.side = Background._streams[key]
        self.pending = False

    def run(self, fn):
        self.side.wait_stream(self.main)
        with torch.cuda.stream(self.side):
            fn()
        self.pending = True

    def join(self):
        if self.pending:
            self.main.wait_stream(self.side)
            self.pending = False


def wgrad(a: torch.Tensor, b: torch.Tensor, colsum: bool = False, out: Optional[torch.Tensor] = None,
          acc: bool = False, max_grid: int = 0, cs_out: Optional[torch.Tensor] = None):
    """Weight gradient ``a^T @ b`` over a long row dimension (K = T*B rows):
    ``a [K, M], b [K, N] -> [M, N]`` (or batched ``[n, K, *] -> [n, M, N]``),
    fp32 output. ``colsum``: also return the column sums of ``b`` (a bias
    gradient that rides on the same pass over ``b``): ``(out, colsum)``.
    ``out``: a contiguous fp32 destination (e.g. :func:`grad_slot`), used by
    the hand-written kernel path. ``acc``: add into ``out`` (and ``cs_out``,
    the colsum destination) instead of overwriting -- row chunks of one
    product summed in a fixed order. ``max_grid`` (a multiple of 8): at most
    that many workgroups, each walking several output tiles (background
    launches beside the recurrent scan); both need the hand-written kernel.

    bf16 operands on the GPU run the hand-written MFMA kernel
    (csrc/wgrad_gemm.hip: 256 x 256 tiles, ds_read_b64_tr_b16 operands,
    split-K only to fill the chip). Other dtypes / shapes use hipBLASLt:
    when the output has few 256x256 tiles K is split S ways into one batched
    product whose partial outputs are summed (measured on MI355X,
    scripts/bench_wgrad.py: the encoder's two [512 x 2048] gradients over
    25000 rows took 168 us at S = 10 against 285 us as a plain batched GEMM)."""
    if a.dtype != b.dtype:
        a, b = a.to(_BF16), b.to(_BF16)
    batched = a.dim() == 3
    if not batched:
        a, b = a.unsqueeze(0), b.unsqueeze(0)
    if _wgrad_hip_ok(a, b):
        out, cs = _wgrad_hip(a, b, colsum, out, acc, max_grid, cs_out)
        if not batched:
            out, cs = out[0], (cs[0] if cs is not None else None)
        return (out, cs) if colsum else out
    if acc or max_grid:
        raise ValueError("wgrad: acc / max_grid need the hand-written bf16 kernel (shape or dtype not taken)")
    if colsum:   # ones column appended to a: the extra output row is colsum(b)
        ones = torch.ones(a.shape[:-1] + (8,), device=a.device, dtype=a.dtype)
        a = torch.cat([a, ones], -1)
    n, K, M = a.shape
    N = b.shape[-1]
    tiles = n * -(-M // 256) * -(-N // 256)
    S = 1
    if a.is_cuda:
        for s in (2, 4, 5, 8, 10, 16, 20, 25, 40, 50):
            if K % s == 0 and K // s >= 512 and tiles * s <= 400:
                S = s
    if S == 1:
        out = bmm(a.transpose(1, 2), b)
    else:
        out = bmm(a.reshape(n * S, K // S, M).transpose(1, 2), b.reshape(n * S, K // S, N))
        out = out.view(n, S, M, N).sum(1)
    cs = None
    if colsum:
        out, cs = out[:, :M - 8], out[:, M - 8]
    if not batched:
        out, cs = out[0], (cs[0] if cs is not None else None)
    return (out, cs) if colsum else out


_SPLITS = (1, 2, 4, 8, 16, 32)  # powers of two: the cell kernels sum <= 8 slabs unrolled


def row_blocks(M: int) -> int:
    """128-row blocks the skinny kernels run for M rows (0: not supported):
    M <= 128 in one block, else ceil(M / 128) blocks up to 1024 rows (the
    grouped kernels take a partial last block; :func:`rec_gemm` routes such
    a product through them)."""
    if M <= 128:
        return 1
    return -(-M // 128) if M <= 1024 else 0


# fp32 operands (fp32 parity runs) through the fp32 MFMA skinny kernel
# (csrc/skinny_gemm.hip skr_skinny_gemm_f32); False: library GEMMs (tests).
F32_GEMM = True


def plan_splits(M: int, N: int, K: int, batch: int = 1, dtype: torch.dtype = _BF16, max_splits: int = 32) -> int:
    """Split-K factor for :func:`rec_gemm`: aim for 256-512 workgroups.
    Returns 0 when the native skinny kernel cannot take the shape."""
    mb = row_blocks(M)
    kt = 64 if dtype == _BF16 else 32            # K-tile of the bf16 / fp32 ring
    if dtype not in (_BF16, torch.float32) or (dtype == torch.float32 and not F32_GEMM):
        return 0
    if mb == 0 or (mb > 1 and batch > 1) or N % 64 or K % kt:
        return 0
    if M > 128 and M % 128 and dtype != _BF16:   # (partial row blocks: the bf16 grouped kernel only)
        return 0
    tiles = (N // 64) * batch * mb
    best = 1
    for s in _SPLITS:
        if s > max_splits or (K // kt) % s:
            continue
        if tiles * s > 512:
            break
        best = s
        if tiles * s >= 256:
            break
    return best


# Skinny products with A in registers (csrc/glds_mma.h ra_mma: only B through
# the LDS-DMA ring): 0 off, else the ring depth (3, 4, 6). Applies to the
# plain and grouped launches (rec_gemm, rec_gemm_group); bit-identical, and
# measured slower (25.5 vs 24.0 ms/step, profiles/r6/skinny_ra_ab.log): off.
SKINNY_RA = 0
_RA_SET = [0]


def _apply_ra(lib) -> None:
    if SKINNY_RA != _RA_SET[0]:
        lib.lib.skr_gemm_set_ra(int(SKINNY_RA))
        _RA_SET[0] = SKINNY_RA


def rec_gemm(a: torch.Tensor, bt: torch.Tensor, out: torch.Tensor, splits: int, nd: int = 1,
             bn: int = 0) -> torch.Tensor:
    """Per-step recurrent product with split-K partial slabs.

    ``a [nd*M, K]`` (row stride may exceed K), ``bt [nd, N, K]`` (B^T, i.e.
    K-contiguous), ``out [S, nd*M, N]`` fp32 with ``S = max(splits, 1)``:
    ``sum_s out[s] = a @ bt^T``. ``splits == 0`` selects the library path
    (one slab). The fused cell kernels sum the slabs while loading.
    """
    M = a.shape[0] // nd
    N, K = bt.shape[-2], bt.shape[-1]
    if splits <= 0 or not a.is_cuda:
        if nd == 1:
            mm(a, bt.reshape(N, K).t(), out=out[0])
        else:
            bmm(a.reshape(nd, M, K), bt.transpose(1, 2), out=out[0].view(nd, M, N))
        return out
    from ..utils import native
    lib = native.require_hip()
    _apply_ra(lib)
    if a.dtype == torch.float32:   # fp32 ring: same arguments, no N-tile choice
        f32 = lib.lib.skr_skinny_gemm_f32
        fn = lambda *args: f32(*args[:-2], args[-1])   # noqa: E731  (drop bn)
    else:
        fn = lib.lib.skr_skinny_gemm_v2
    if nd == 1 and M > 128 and M % 128:   # a partial last row block: the grouped kernel takes it
        _launch_group([(a, bt, out, splits)])
        return out
    if nd == 1 and M > 128:   # 128-row blocks as the kernel's batch dimension, sharing B
        mb = row_blocks(M)
        rc = fn(a.data_ptr(), a.stride(0), 128 * a.stride(0), bt.data_ptr(), bt.stride(-2), 0, out.data_ptr(), N,
                out.stride(0), 128 * N, 128, N, K, splits, mb, bn, torch.cuda.current_stream().cuda_stream)
    else:
        rc = fn(a.data_ptr(), a.stride(0), M * a.stride(0), bt.data_ptr(), bt.stride(-2), N * K if nd > 1 else 0,
                out.data_ptr(), N, out.stride(0), M * N, M, N, K, splits, nd, bn,
                torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_skinny_gemm failed (%d) for M=%d N=%d K=%d S=%d" % (rc, M, N, K, splits))
    return out


def rec_gemm_bf16out(a: torch.Tensor, bt: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """``out [M, N] (bf16) = a @ bt^T`` in one slab (no split-K): for products
    read only as bf16 downstream (csrc/skinny_gemm.hip ``skr_skinny_gemm_v2_bf16out``)."""
    from ..utils import native
    lib = native.require_hip()
    M, K = a.shape
    N = bt.shape[-2]
    assert out.dtype == _BF16 and out.shape[-1] == N and M <= 128
    rc = lib.lib.skr_skinny_gemm_v2_bf16out(a.data_ptr(), a.stride(0), 0, bt.data_ptr(), bt.stride(-2), 0,
                                            out.data_ptr(), out.stride(-2), 0, M, N, K, 1,
                                            torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_skinny_gemm_v2_bf16out failed (%d) for M=%d N=%d K=%d" % (rc, M, N, K))
    return out


GROUPED = os.environ.get("SKR_GEMM_GROUP", "1") != "0"   # SKR_GEMM_GROUP=0: independent per-step products as separate launches


# N-tile width of the grouped launch (0: the kernel's default, 64; 128: 8-wave
# tiles, measured slower -- profiles/r5/bench_group.jsonl); sweeps set it
GROUP_BN = 0


def rec_gemm_group(jobs) -> None:
    """Several independent :func:`rec_gemm` products ``(a, bt, out, splits)``
    (nd = 1, bf16, splits >= 1; M <= 128, or 128-row blocks up to 1024) in
    ONE grouped launch
    (csrc/skinny_gemm.hip ``skr_skinny_gemm_group``); falls back to one
    launch per product when a job does not qualify."""
    ok = GROUPED and 1 <= len(jobs) <= 4 and all(
        a.is_cuda and a.dtype == _BF16 and s >= 1 and row_blocks(a.shape[0]) > 0 for a, _, _, s in jobs)
    if not ok:
        for a, bt, out, s in jobs:
            rec_gemm(a, bt, out, s)
        return
    _launch_group(jobs)


def _launch_group(jobs) -> None:
    from ..utils import native
    from ._hipapi import GemmProblem
    lib = native.require_hip()
    _apply_ra(lib)
    probs = (GemmProblem * len(jobs))()
    for p, (a, bt, out, s) in zip(probs, jobs):
        N, K = bt.shape[-2], bt.shape[-1]
        p.A, p.lda, p.Bt, p.ldb = a.data_ptr(), a.stride(0), bt.data_ptr(), bt.stride(-2)
        p.C, p.ldc, p.c_slab = out.data_ptr(), N, out.stride(0)
        p.M, p.N, p.K, p.splits = a.shape[0], N, K, s
    rc = lib.lib.skr_skinny_gemm_group(probs, len(jobs), GROUP_BN, torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_skinny_gemm_group failed (%d)" % rc)


def _problems(jobs):
    from ._hipapi import GemmProblem
    probs = (GemmProblem * len(jobs))()
    for p, (a, bt, out, s) in zip(probs, jobs):
        assert a.is_cuda and a.dtype == _BF16 and s >= 1 and a.shape[0] <= 1024
        N, K = bt.shape[-2], bt.shape[-1]
        p.A, p.lda, p.Bt, p.ldb = a.data_ptr(), a.stride(0), bt.data_ptr(), bt.stride(-2)
        p.C, p.ldc, p.c_slab = out.data_ptr(), N, out.stride(0)
        p.M, p.N, p.K, p.splits = a.shape[0], N, K, s
    return probs


def rec_gemm_group_cellbwd(jobs, cell_args) -> None:
    """:func:`rec_gemm_group` products plus one backward LayerNorm cell step
    (``cell_args``: a filled ``LstmBwdArgs``, one workgroup per row, H <= 256)
    in ONE launch (``skr_skinny_gemm_group_cellbwd``): the cell rows run
    beside the GEMM tiles."""
    import ctypes
    from ..utils import native
    lib = native.require_hip()
    probs = _problems(jobs)
    rc = lib.lib.skr_skinny_gemm_group_cellbwd(probs, len(jobs), ctypes.byref(cell_args),
                                               torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_skinny_gemm_group_cellbwd failed (%d)" % rc)


# ---- chained launches (csrc/chain_step.hip) ----------------------------------------------
class ChainCounters:
    """Rotating arrival counters of one chained launch kind over a sequence
    of ``n`` launches (launch ``k`` uses counter ``k`` and zeroes counter
    ``k + 1``): zero-initialised once (normally in the eager warm-up, so no
    fill kernel lands in a captured step), cached per (device, kind, n) so a
    captured HIP graph keeps replaying on the same words. Sequences of one
    kind must not run concurrently on different streams."""
    _cache = {}

    def __init__(self, device, kind: str, n: int):
        from .recurrent import cluster_error_flag
        from ._hipapi import ChainSync
        key = (str(device), kind, n)
        buf = ChainCounters._cache.get(key)
        if buf is None:
            buf = ChainCounters._cache[key] = torch.zeros(max(n, 2), dtype=torch.int32, device=device)
        self.buf, self.n = buf, n
        self.sync = ChainSync()
        self.sync.counters, self.sync.n, self.sync.err = buf.data_ptr(), n, cluster_error_flag(device).data_ptr()

    def at(self, k: int):
        self.sync.k = k
        return self.sync


def chain_bwd_main(producers, cell_args, sync) -> int:
    """One launch: ``producers`` feeding the HyperLSTM main cell's dh_rec
    slabs and the main-cell backward rows (``skr_chain_bwd_main``, H = 2048).
    Returns the library code: -2 / -3 / -4 mean "shape not taken" (the caller
    falls back to the unchained launches)."""
    import ctypes
    from ..utils import native
    lib = native.require_hip()
    rc = lib.lib.skr_chain_bwd_main(_problems(producers), len(producers), ctypes.byref(cell_args), ctypes.byref(sync),
                                    torch.cuda.current_stream().cuda_stream)
    if rc not in (0, -2, -3, -4):
        raise RuntimeError("skr_chain_bwd_main failed (%d)" % rc)
    return rc


def chain_bwd_main3(producers, tail, cell_args, sync, rows_sync) -> int:
    """:func:`chain_bwd_main` plus the ``tail`` product ``(dvec, P^T, out,
    splits)`` in the SAME launch (``skr_chain_bwd_main3``): the first producer
    workgroups, once their producer tile is done, stage their P^T weight slice
    in LDS while the main-cell rows compute, then run the dvec P^T tile on the
    rows' arrival counters ``rows_sync``. Returns the library code (-2 / -3 /
    -4: not taken, the caller keeps the separate launches)."""
    import ctypes
    from ..utils import native
    lib = native.require_hip()
    rc = lib.lib.skr_chain_bwd_main3(_problems(producers), len(producers), _problems([tail]), ctypes.byref(cell_args),
                                     ctypes.byref(sync), ctypes.byref(rows_sync), torch.cuda.current_stream().cuda_stream)
    if rc not in (0, -2, -3, -4):
        raise RuntimeError("skr_chain_bwd_main3 failed (%d)" % rc)
    return rc


def chain_ln_fwd(producers, cell_args, sync) -> int:
    """One launch: ``producers`` writing the R slabs of a LayerNorm-LSTM step
    and that step's forward cell rows (``skr_chain_ln_fwd``). Returns the
    library code: -2 / -3 / -4 mean "shape not taken"."""
    import ctypes
    from ..utils import native
    lib = native.require_hip()
    rc = lib.lib.skr_chain_ln_fwd(_problems(producers), len(producers), ctypes.byref(cell_args), ctypes.byref(sync),
                                  torch.cuda.current_stream().cuda_stream)
    if rc not in (0, -2, -3, -4):
        raise RuntimeError("skr_chain_ln_fwd failed (%d)" % rc)
    return rc


def chain_ln_bwd(producers, cell_args, sync) -> int:
    """One launch: ``producers`` writing the dh slabs of a LayerNorm-LSTM
    backward step and that step's cell backward rows (``skr_chain_ln_bwd``).
    Returns the library code: -2 / -3 / -4 mean "shape not taken"."""
    import ctypes
    from ..utils import native
    lib = native.require_hip()
    rc = lib.lib.skr_chain_ln_bwd(_problems(producers), len(producers), ctypes.byref(cell_args), ctypes.byref(sync),
                                  torch.cuda.current_stream().cuda_stream)
    if rc not in (0, -2, -3, -4):
        raise RuntimeError("skr_chain_ln_bwd failed (%d)" % rc)
    return rc


# ---- inference-time helpers ------------------------------------------------------------
_WCACHE = {}
WEIGHTS_EPOCH = [0]


def invalidate_derived() -> None:
    """Drop cached inference weight copies. Called by every code path that
    changes parameters without bumping their version counters -- optimizer
    steps replayed from a HIP graph, checkpoint loads."""
    _WCACHE.clear()
    WEIGHTS_EPOCH[0] += 1


def derived(W, tag: str, fn):
    """``fn(W)`` cached while ``W`` (a tensor or a tuple of tensors) is
    unchanged (same storage and version): for inference, so per-call weight
    casts / transposes / quantisation run once instead of at every decode
    step. Parameter updates replayed from a HIP graph do not bump version
    counters: the trainers call :func:`invalidate_derived` every step."""
    ws = W if isinstance(W, tuple) else (W,)
    key = (tag,) + tuple((w.data_ptr(), w._version, tuple(w.shape), w.dtype) for w in ws)
    hit = _WCACHE.get(key)
    # the entry holds its source tensors: a freed-and-reallocated tensor at the
    # same address (fresh version counter) is a different object -> miss
    if hit is not None and all(a is b for a, b in zip(hit[0], ws)):
        return hit[1]
    if len(_WCACHE) > 512:
        _WCACHE.clear()
    v = fn(*ws)
    _WCACHE[key] = (ws, v)
    return v


def cast_transpose(W: torch.Tensor, plain: Optional[torch.Tensor] = None, trans: Optional[torch.Tensor] = None,
                   want_plain: bool = True, want_trans: bool = True):
    """fp32 ``W [..., R, C]`` -> bf16 ``W`` and bf16 ``W^T [..., C, R]`` in one
    pass (csrc/convert.hip). ``plain`` / ``trans`` may be given (views into
    larger buffers: row-strided, e.g. a column slice of a concatenated B^T);
    returns ``(plain, trans)``. CPU tensors / fp32 compute: torch ops."""
    R, C = W.shape[-2], W.shape[-1]
    nb = W.numel() // (R * C) if W.numel() else 0
    lead = W.shape[:-2]
    if plain is None and want_plain:
        plain = torch.empty(*lead, R, C, dtype=_BF16, device=W.device)
    if trans is None and want_trans:
        trans = torch.empty(*lead, C, R, dtype=_BF16, device=W.device)
    Wc = W.detach()
    sb = lambda t: (t.stride(-3) if t.dim() >= 3 else 0) if t is not None else 0   # noqa: E731
    # the kernel's vector loads / stores need rows (and batches) in multiples of 4 elements
    vec_ok = all(t is None or (t.stride(-1) == 1 and t.stride(-2) % 4 == 0 and sb(t) % 4 == 0
                               and t.data_ptr() % (16 if t is Wc else 8) == 0) for t in (Wc, plain, trans))
    if not Wc.is_cuda or Wc.dtype != torch.float32 or not vec_ok:
        if plain is not None:
            plain.copy_(Wc)
        if trans is not None:
            trans.copy_(Wc.transpose(-1, -2))
        return plain, trans
    from ..utils import native
    lib = native.require_hip()
    rc = lib.lib.skr_cast_transpose_bf16(
        Wc.data_ptr(), Wc.stride(-2), sb(Wc), R, C, max(nb, 1),
        plain.data_ptr() if plain is not None else None, plain.stride(-2) if plain is not None else 0, sb(plain),
        trans.data_ptr() if trans is not None else None, trans.stride(-2) if trans is not None else 0, sb(trans),
        torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError("skr_cast_transpose_bf16 failed (%d) for %s" % (rc, tuple(W.shape)))
    return plain, trans


class _Linear(torch.autograd.Function):
    """``x @ W + b`` in the compute precision with fp32 outputs/grads."""

    @staticmethod
    def forward(ctx, x, W, b):
        xs = x.reshape(-1, x.shape[-1])
        xl, Wl = lp(xs), lp(W)
        y = mm(xl, Wl)
        if b is not None:
            y.add_(b)
        ctx.save_for_backward(xl, Wl)
        ctx.has_b = b is not None
        ctx.shape = x.shape
        return y.view(*x.shape[:-1], W.shape[1])

    @staticmethod
    def backward(ctx, dy):
        xl, Wl = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dyl = lp(dy2)
        dx = dW = db = None
        if ctx.needs_input_grad[0]:
            dx = mm(dyl, Wl.t()).view(ctx.shape)
        if ctx.needs_input_grad[1]:
            dW = wgrad(xl, dyl)
        if ctx.has_b and ctx.needs_input_grad[2]:
            from .reduce import colsum
            db = colsum(dy2)[1]   # torch's dim-0 sum is ~0.35 ms on [25000, 123]
        return dx, dW, db


def linear(x: torch.Tensor, W: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    if lp_dtype() == torch.float32 or not x.is_cuda:
        y = x.reshape(-1, x.shape[-1]) @ W
        if b is not None:
            y = y + b
        return y.view(*x.shape[:-1], W.shape[1])
    if not (torch.is_grad_enabled() and (x.requires_grad or W.requires_grad)):
        # inference: the low-precision weight copy is made once, not per call
        y = mm(lp(x.reshape(-1, x.shape[-1])), derived(W, "lp%s" % lp_dtype(), lp))
        if b is not None:
            y.add_(b)
        return y.view(*x.shape[:-1], W.shape[1])
    return _Linear.apply(x, W, b)
