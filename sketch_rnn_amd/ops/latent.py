"""The VAE latent layer as one autograd node (``csrc/latent.hip``).

``latent(h, W_mu, b_mu, W_sig, b_sig, W_init, b_init, seed, widths)``:

    mu = h W_mu + b_mu,  presig = h W_sig + b_sig
    z  = mu + exp(presig / 2) eps            eps = hash normal (seed, stream, step 0), or given
    kl = max(-0.5 mean(1 + presig - mu^2 - exp(presig)), kl_tolerance)
    s  = tanh(z W_init + b_init) split column-wise into ``widths``

returns ``(mu, presig, z, kl, *segments)``. Reference semantics: the magenta
sketch_rnn encoder head / reparameterisation / KL and the decoder's initial
state (our torch form: models/vae.py ``SketchVAE.loss``). The three GEMMs and
their gradients run on csrc/small_gemm.hip (bias fused); everything between them is two small
kernels forward and two backward instead of ~35 elementwise launches.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from ..utils import native
from .gemm import SmallGroup, small_mm
from .reduce import colsum_many


def latent_ok(h: torch.Tensor, n_seg: int) -> bool:
    from . import use_hip
    return h.is_cuda and use_hip(h) and 1 <= n_seg <= 4 and h.dtype == torch.float32


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() if t is not None else None for t in ts])


class _Latent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, w_mu, b_mu, w_sig, b_sig, w_init, b_init, seed, eps, meta):
        widths, kl_tol, stream = meta
        ctx.set_materialize_grads(False)   # mu / presig are usually unused: None grads
        lib = native.require_hip().lib
        st = torch.cuda.current_stream().cuda_stream
        h = h.contiguous()
        g = SmallGroup(h.device)   # the two heads in one launch
        mu = g.mm(h, w_mu, b_mu)
        ps = g.mm(h, w_sig, b_sig)
        g.run()
        B, Z = mu.shape
        dev = h.device
        z = torch.empty(B, Z, device=dev)
        ep = torch.empty(B, Z, device=dev)
        kl_raw = torch.empty((), device=dev)
        kl = torch.empty((), device=dev)
        eps_c = eps.contiguous().float() if eps is not None else None
        rc = lib.skr_latent_mid(mu.data_ptr(), ps.data_ptr(), eps_c.data_ptr() if eps_c is not None else None,
                                seed.data_ptr(), stream, B * Z, float(kl_tol), z.data_ptr(), ep.data_ptr(),
                                kl_raw.data_ptr(), kl.data_ptr(), st)
        if rc != 0:
            raise RuntimeError("skr_latent_mid failed (%d)" % rc)
        pre = small_mm(z, w_init, b_init)
        S = pre.shape[1]
        segs = [torch.empty(B, w, device=dev) for w in widths]
        wa = (ctypes.c_int * len(widths))(*widths)
        rc = lib.skr_tanh_split(pre.data_ptr(), B, S, len(widths), wa, _ptrs(segs), st)
        if rc != 0:
            raise RuntimeError("skr_tanh_split failed (%d)" % rc)
        ctx.save_for_backward(h, mu, ps, ep, z, kl_raw, w_mu, w_sig, w_init, *segs)
        ctx.meta = meta
        return (mu, ps, z, kl, *segs)

    @staticmethod
    def backward(ctx, dmu, dps, dz, dkl, *dsegs):
        widths, kl_tol, stream = ctx.meta
        h, mu, ps, ep, z, kl_raw, w_mu, w_sig, w_init, *segs = ctx.saved_tensors
        lib = native.require_hip().lib
        st = torch.cuda.current_stream().cuda_stream
        B, Z = mu.shape
        S = w_init.shape[1]
        dev = h.device
        dsegs = [g.contiguous() if g is not None else None for g in dsegs]
        dpre = torch.empty(B, S, device=dev)
        wa = (ctypes.c_int * len(widths))(*widths)
        rc = lib.skr_tanh_split_bwd(B, S, len(widths), wa, _ptrs(segs), _ptrs(dsegs), dpre.data_ptr(), st)
        if rc != 0:
            raise RuntimeError("skr_tanh_split_bwd failed (%d)" % rc)
        g = SmallGroup(dev)
        dW_init = g.mm(z.t(), dpre)
        dz_int = g.mm(dpre, w_init.t())
        g.run()
        dmu_t = torch.empty(B, Z, device=dev)
        dps_t = torch.empty(B, Z, device=dev)
        c = lambda t: t.contiguous() if t is not None else None   # noqa: E731
        dz, dmu, dps, dkl = c(dz), c(dmu), c(dps), c(dkl)
        p = lambda t: t.data_ptr() if t is not None else None     # noqa: E731
        rc = lib.skr_latent_mid_bwd(mu.data_ptr(), ps.data_ptr(), ep.data_ptr(), kl_raw.data_ptr(), float(kl_tol),
                                    p(dkl), dz_int.data_ptr(), p(dz), p(dmu), p(dps), B * Z, dmu_t.data_ptr(),
                                    dps_t.data_ptr(), st)
        if rc != 0:
            raise RuntimeError("skr_latent_mid_bwd failed (%d)" % rc)
        g = SmallGroup(dev)
        dh = g.mm(dmu_t, w_mu.t())
        dW_mu = g.mm(h.t(), dmu_t)
        dW_sig = g.mm(h.t(), dps_t)
        g.run()
        small_mm(dps_t, w_sig.t(), out=dh, acc=True)
        (_, db_init), (_, db_mu), (_, db_sig) = colsum_many([(dpre, None), (dmu_t, None), (dps_t, None)])
        return dh, dW_mu, db_mu, dW_sig, db_sig, dW_init, db_init, None, None, None


def latent(h, w_mu, b_mu, w_sig, b_sig, w_init, b_init, seed: torch.Tensor, widths: Sequence[int],
           kl_tolerance: float, stream: int, eps: Optional[torch.Tensor] = None):
    """See the module docstring. ``seed``: device int64 tensor (graph-safe)."""
    return _Latent.apply(h, w_mu, b_mu, w_sig, b_sig, w_init, b_init, seed, eps,
                         (tuple(int(w) for w in widths), float(kl_tolerance), int(stream)))
