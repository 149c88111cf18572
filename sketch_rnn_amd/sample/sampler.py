"""Sketch generation.

Host samplers (exact semantics, any device, one sketch at a time):

* :func:`sample_reference` -- the reference's ``Model.sample``
  (``model.py:187-264``): zero first input, mixture temperature applied from
  step 2 on, inverse-CDF draws with the "-1 -> last component" rule, sigma
  NOT temperature-scaled, optional early stop on ``eoc`` (the ``eoc`` row is
  kept), offsets multiplied by ``data_scale``. The reference's pen-temperature
  bug (``pi_pdf /= temp_pen``, ``model.py:230``) is reproduced by default;
  ``fix_pen_temperature=True`` applies the temperature to the pen logits.
* :func:`sample_vae` -- sketch-rnn VAE semantics: start token
  ``[0, 0, 1, 0, 0]``, temperature on mixture and pen, sigma scaled by the
  temperature, optional greedy mode, ``z`` from N(0, I) or given.

Device sampler (:class:`GraphDecoder`): B sketches in parallel, the
N-step decode loop (decoder step -> MDN head -> ``csrc/sampler.hip``, which
writes the next input on device) captured once into a HIP graph and
replayed; finished rows emit end-of-sketch padding. No host round trip per
stroke (the reference does two ``sess.run`` transfers per stroke). HyperLSTM
decoders step through :class:`~.hyper_step.HyperStepDecoder` (state in
place, seven hand-written kernels per stroke); the reference model has a
one-launch whole-sketch decoder in :mod:`.fused`.
"""
from __future__ import annotations

import math
import os
import random as _random
from typing import List, Optional, Tuple

import numpy as np
import torch

from ..models import mdn as M
from ..train.graph import capture


def _get_pi_idx(x: float, pdf: np.ndarray) -> int:
    acc = 0.0
    for i in range(pdf.size):
        acc += pdf[i]
        if acc >= x:
            return i
    return -1


def _softmax_np(v):
    v = np.asarray(v, dtype=np.float64)
    v = v - v.max()
    e = np.exp(v)
    return e / e.sum()


@torch.no_grad()
def sample_reference(model, num: int = 300, temp_mixture: float = 1.0, temp_pen: float = 1.0,
                     stop_if_eoc: bool = False, rng: Optional[np.random.RandomState] = None,
                     py_rng: Optional[_random.Random] = None, fix_pen_temperature: bool = False,
                     device=None):
    """Reference ``Model.sample``. Returns ``(strokes [n, 5], mixture_params)``."""
    rng = rng or np.random.RandomState()
    py_rng = py_rng or _random.Random()
    cfg = model.cfg
    dev = device or next(model.parameters()).device
    Mx = cfg.num_mixture
    prev_x = torch.zeros(1, 5, device=dev)
    state = model.zero_state(1, dev)
    strokes = np.zeros((num, 5), dtype=np.float32)
    params = []
    for i in range(num):
        z, next_state = model.step(prev_x, state)
        pi, mu1, mu2, s1, s2, rho, _, pen_logits = (t[0].double().cpu().numpy() for t in M.mixture_coef(z, Mx))
        pi_pdf = pi.copy()
        if i > 1:
            pi_pdf = np.log(pi_pdf) / temp_mixture
            pi_pdf -= pi_pdf.max()
            pi_pdf = np.exp(pi_pdf)
        pi_pdf /= pi_pdf.sum()
        idx = _get_pi_idx(py_rng.random(), pi_pdf)
        pen = pen_logits.copy()
        if i > 1:
            if fix_pen_temperature:
                pen = pen / temp_pen
            else:
                pi_pdf /= temp_pen  # reference bug: rescales pi, pen temperature has no effect
        pen_pdf = _softmax_np(pen)
        pen_idx = _get_pi_idx(py_rng.random(), pen_pdf)
        eos, eoc, cont = (1, 0, 0) if pen_idx == 0 else (0, 1, 0) if pen_idx == 1 else (0, 0, 1)
        cov = [[s1[idx] ** 2, rho[idx] * s1[idx] * s2[idx]], [rho[idx] * s1[idx] * s2[idx], s2[idx] ** 2]]
        x1, x2 = rng.multivariate_normal([mu1[idx], mu2[idx]], cov, 1)[0]
        strokes[i] = [x1, x2, eos, eoc, cont]
        params.append([pi_pdf, mu1, mu2, s1, s2, rho, pen_pdf])
        if stop_if_eoc and eoc == 1:
            strokes = strokes[: i + 1]
            break
        prev_x = torch.tensor([[x1, x2, eos, eoc, cont]], dtype=torch.float32, device=dev)
        state = next_state
    strokes[:, 0:2] *= cfg.data_scale
    return strokes, params


def _adjust_temp(pdf: np.ndarray, temp: float) -> np.ndarray:
    p = np.log(pdf) / temp
    p -= p.max()
    p = np.exp(p)
    return p / p.sum()


@torch.no_grad()
def sample_vae(model, seq_len: int = 250, temperature: float = 1.0, greedy: bool = False,
               z: Optional[torch.Tensor] = None, label: Optional[int] = None,
               rng: Optional[np.random.RandomState] = None, py_rng: Optional[_random.Random] = None):
    """One sketch from the VAE decoder. Returns ``(strokes5 [seq_len, 5], params)``
    in the magenta layout (convert with ``data.strokes.to_normal_strokes``)."""
    rng = rng or np.random.RandomState()
    py_rng = py_rng or _random.Random()
    cfg = model.cfg
    dev = next(model.parameters()).device
    if cfg.conditional and z is None:
        z = torch.as_tensor(rng.randn(1, cfg.z_size), dtype=torch.float32, device=dev)
    lab = torch.tensor([label], device=dev) if (label is not None and cfg.num_classes > 0) else None
    zc = model.condition(z if cfg.conditional else None, lab, 1, dev)
    state = model.initial_state(zc, 1, dev)
    prev_x = torch.tensor([[0.0, 0.0, 1.0, 0.0, 0.0]], device=dev)
    strokes = np.zeros((seq_len, 5), dtype=np.float32)
    params = []
    for i in range(seq_len):
        zh, state = model.decode_step(prev_x, zc, state)
        pi, mu1, mu2, s1, s2, rho, pen, _ = (t[0].double().cpu().numpy() for t in M.mixture_coef(zh, cfg.num_mixture))
        if greedy:
            idx, pidx = int(np.argmax(pi)), int(np.argmax(pen))
            x1, x2 = mu1[idx], mu2[idx]
        else:
            idx = _get_pi_idx(py_rng.random(), _adjust_temp(pi, temperature))
            pidx = _get_pi_idx(py_rng.random(), _adjust_temp(pen, temperature))
            sa, sb = s1[idx] * temperature, s2[idx] * temperature
            cov = [[sa * sa, rho[idx] * sa * sb], [rho[idx] * sa * sb, sb * sb]]
            x1, x2 = rng.multivariate_normal([mu1[idx], mu2[idx]], cov, 1)[0]
        row = [x1, x2, 0.0, 0.0, 0.0]
        row[2 + pidx] = 1.0
        strokes[i] = row
        params.append([pi, mu1, mu2, s1, s2, rho, pen])
        prev_x = torch.tensor([row], dtype=torch.float32, device=dev)
    return strokes, params


# =====================================================================================
# device sampler + HIP graph decode
# =====================================================================================
_SAMPLE_STREAM = 0x5A3D
# GraphDecoder steps VAE decoders with the in-place step decoders
# (sample/hyper_step.py) where they apply; False: the generic decode_step.
STEP_DECODER = os.environ.get("SKR_STEP_DECODER", "1") != "0"


def mdn_sample_torch(zh: torch.Tensor, M_: int, mode: int, temp: float, greedy: bool, fix_pen: bool,
                     seed, step: int, out_row: torch.Tensor, next_x: torch.Tensor, done: torch.Tensor,
                     params: Optional[torch.Tensor] = None) -> None:
    """PyTorch transcription of ``csrc/sampler.hip`` (same hash random
    numbers, same draws): the CPU path of :class:`GraphDecoder` and the
    oracle the kernel is tested against."""
    from ..models.cells import hash_uniform
    B = zh.shape[0]
    z = zh.float()
    u = hash_uniform(seed, _SAMPLE_STREAM, step, (B, 4), device=z.device)
    use_t = mode == 1 or step > 1
    logits = z[:, 3:3 + M_] * ((1.0 / temp) if use_t else 1.0)
    pi = torch.softmax(logits, -1)
    ar = torch.arange(B, device=z.device)
    if greedy:
        idx = pi.argmax(-1)
    else:
        hit = torch.cumsum(pi, -1) >= u[:, 0:1]
        idx = torch.where(hit.any(-1), hit.float().argmax(-1), torch.full_like(ar, M_ - 1))
    pt = (1.0 / temp) if (mode == 1 or (fix_pen and step > 1)) else 1.0
    pp = torch.softmax(z[:, 0:3] * pt, -1)
    if greedy:
        pidx = pp.argmax(-1)
    else:
        hit = torch.cumsum(pp, -1) >= u[:, 1:2]
        pidx = torch.where(hit.any(-1), hit.float().argmax(-1), torch.full_like(ar, 2))
    col = lambda k: z[ar, 3 + k * M_ + idx]  # noqa: E731
    mu1, mu2, s1, s2, rho = col(1), col(2), torch.exp(col(3)), torch.exp(col(4)), torch.tanh(col(5))
    if mode == 1:
        s1, s2 = s1 * temp, s2 * temp
    x1, x2 = mu1, mu2
    if not greedy:
        r = torch.sqrt(-2.0 * torch.log(torch.clamp(u[:, 2], min=1e-12)))
        n1, n2 = r * torch.cos(2 * math.pi * u[:, 3]), r * torch.sin(2 * math.pi * u[:, 3])
        x1 = mu1 + s1 * n1
        x2 = mu2 + s2 * (rho * n1 + torch.sqrt(torch.clamp(1 - rho * rho, min=0.0)) * n2)
    row = torch.zeros(B, 5, device=z.device)
    row[:, 0], row[:, 1] = x1, x2
    row[ar, 2 + pidx] = 1.0
    stop_col = 4 if mode == 1 else 3
    pad = torch.zeros(B, 5, device=z.device)
    pad[:, stop_col] = 1.0
    out_row.copy_(torch.where((done != 0).unsqueeze(-1), pad, row))
    next_x.copy_(row)
    done.copy_(torch.where(pidx + 2 == stop_col, torch.ones_like(done), done))
    if params is not None:
        params.copy_(torch.stack([idx.float(), pidx.float(), s1, s2], -1))


def mdn_sample_device(zh: torch.Tensor, M_: int, mode: int, temp: float, greedy: bool, fix_pen: bool,
                      seed: torch.Tensor, step: int, out_row: torch.Tensor, next_x: torch.Tensor,
                      done: torch.Tensor, params: Optional[torch.Tensor] = None) -> None:
    if zh.device.type != "cuda":
        return mdn_sample_torch(zh, M_, mode, temp, greedy, fix_pen, seed, step, out_row, next_x, done, params)
    assert zh.dtype == torch.float32 and zh.stride(1) == 1 and zh.shape[1] >= 3 + 6 * M_
    assert out_row.dtype == torch.float32 and out_row.stride(-1) == 1 and out_row.shape[0] == zh.shape[0]
    assert next_x.shape == (zh.shape[0], 5) and next_x.stride(-1) == 1
    assert done.dtype == torch.int32 and done.numel() == zh.shape[0] and seed.dtype == torch.int64
    from ..utils import native
    lib = native.require_hip()
    import ctypes
    rc = lib.lib.skr_mdn_sample(ctypes.c_void_p(zh.data_ptr()), ctypes.c_int64(zh.stride(0)), ctypes.c_int(zh.shape[0]),
                                ctypes.c_int(M_), ctypes.c_int(mode), ctypes.c_float(temp), ctypes.c_int(int(greedy)),
                                ctypes.c_int(int(fix_pen)), ctypes.c_void_p(seed.data_ptr()), ctypes.c_uint32(step),
                                ctypes.c_void_p(out_row.data_ptr()), ctypes.c_int64(out_row.stride(0)),
                                ctypes.c_void_p(next_x.data_ptr()), ctypes.c_int64(next_x.stride(0)),
                                ctypes.c_void_p(done.data_ptr()),
                                ctypes.c_void_p(params.data_ptr() if params is not None else 0),
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError("skr_mdn_sample failed (%d)" % rc)


class GraphDecoder:
    """Batched autoregressive decode captured in HIP graphs.

    ``model`` is a :class:`~sketch_rnn_amd.models.reference.SketchRNN` (mode
    ``reference``) or :class:`~sketch_rnn_amd.models.vae.SketchVAE` (mode
    ``vae``). ``run()`` returns ``strokes [B, N, 5]`` (offsets in model
    units; reference mode multiplies by ``data_scale``) plus the per-row
    number of valid steps.

    The N steps are captured as consecutive chunks of ``chunk`` steps, one
    graph each (one memory pool). After each chunk the host reads whether
    every row has drawn its end-of-sketch pen state; if so the remaining
    chunks are skipped and their output rows are filled with the padding
    row the sampler would have emitted (reference: model.py:254-257, the
    ``stop_if_eoc`` break). The emitted sketches are identical to the
    full-length decode: finished rows only ever emit padding, and the
    sampler's noise is keyed by (seed, step, row), not by a running state.
    ``steps_run`` records how many decode steps the last ``run()`` executed.
    """

    CHUNK = 25               # steps per captured graph (one host read of the all-done flag per chunk)

    def __init__(self, model, batch: int, steps: int, temperature: float = 1.0, greedy: bool = False,
                 fix_pen_temperature: bool = False, use_graph: bool = True, chunk: Optional[int] = None,
                 early_exit: bool = True, fp8: bool = False):
        self.model = model
        self.kind = "vae" if hasattr(model, "encoder") else "reference"
        self.B, self.N = batch, steps
        self.temp, self.greedy, self.fix_pen = float(temperature), bool(greedy), bool(fix_pen_temperature)
        dev = next(model.parameters()).device
        self.dev = dev
        cfg = model.cfg
        self.Mx = cfg.num_mixture
        self.mode = 1 if self.kind == "vae" else 0
        self.seed = torch.zeros(1, dtype=torch.int64, device=dev)
        self.out = torch.zeros(batch, steps, 5, device=dev)
        self.done = torch.zeros(batch, dtype=torch.int32, device=dev)
        self.x0 = torch.zeros(batch, 5, device=dev)
        if self.kind == "vae":
            self.x0[:, 2] = 1.0
            self.z = torch.zeros(batch, max(cfg.z_size, 1), device=dev)
            self.labels = torch.zeros(batch, dtype=torch.int64, device=dev)
        self.graphs = None
        self.use_graph = use_graph and dev.type == "cuda"
        c = int(chunk or self.CHUNK)
        self.ranges = [(t, min(t + c, steps)) for t in range(0, steps, c)] if steps > 0 else []
        self.early_exit = bool(early_exit)
        self.fp8 = bool(fp8)   # MX-fp8 h W_h in the HyperLSTM step decoders (BASELINE config 5)
        self.steps_run = 0
        self._carry = {}     # tensors handed from one chunk to the next (state, next input, zc)

    _MAX_CHUNKS = 8          # concurrent 128-row step decoders (one HIP stream each)

    def _steppers(self):
        """Lean in-place HyperLSTM step decoders (``sample/hyper_step.py``), one
        per chunk of <= 128 rows, when the model qualifies; else None.

        Chunks run CONCURRENTLY, one stream each (captured as parallel graph
        branches): each stroke's chain is latency-bound, so a second chain
        fills the idle CUs. Only chunk 0's main cell uses the clustered
        LayerNorm exchange (co-resident spin-waits); the others keep every
        row in one workgroup, so no two spin-waiting launches ever compete
        for residency."""
        if self.kind != "vae" or self.dev.type != "cuda" or not STEP_DECODER:
            return None
        from .hyper_step import HyperStepDecoder, hyper_step_ok, wide_ok
        if self.B > 128 and self.B % 128 == 0 and self.B <= 1024 and wide_ok(self.model):
            chunks = [(0, self.B)]   # one wide decoder: 128-row blocks inside each launch
        else:
            chunks = [(r0, min(128, self.B - r0)) for r0 in range(0, self.B, 128)]
        if len(chunks) > self._MAX_CHUNKS or not all(hyper_step_ok(self.model, n) for _, n in chunks):
            return None
        if getattr(self, "_stp", None) is None:
            # chunk 0 runs on whatever stream is current at decode time (None)
            self._stp = [(r0, n, HyperStepDecoder(self.model, n, self.dev, cluster=(i == 0), fp8=self.fp8),
                          None if i == 0 else torch.cuda.Stream(device=self.dev))
                         for i, (r0, n) in enumerate(chunks)]
        return self._stp

    @torch.no_grad()
    def _decode_steppers(self, stp, t0, t1):
        import ctypes
        from ..utils import native
        lib = native.require_hip().lib
        model, B, N = self.model, self.B, self.N
        cfg = model.cfg
        ld_out = self.out.stride(0)
        main = torch.cuda.current_stream(self.dev)
        stp = [(r0, n, st, main if stream is None else stream) for r0, n, st, stream in stp]
        cy = self._carry
        if t0 == 0:
            lab = self.labels if cfg.num_classes > 0 else None
            cy["zc"] = zc = model.condition(self.z if cfg.conditional else None, lab, B, self.dev)
            cy["state"] = model.initial_state(zc, B, self.dev)
            cy["x0"] = self.x0.clone()
            for _, _, st, _ in stp:              # weight operands on the parent stream
                st.prepare()
        zc, state, x0 = cy["zc"], cy["state"], cy["x0"]
        for _, _, _, stream in stp:              # fork: inputs above are ready
            if stream != main:
                stream.wait_stream(main)
        for i, (r0, n, st, stream) in enumerate(stp):
            if st.fused:       # four launches per stroke (hyper_step.py module docstring)
                with torch.cuda.stream(stream):
                    if t0 == 0:
                        st.begin(zc[r0:r0 + n] if zc is not None else None, [s[r0:r0 + n] for s in state],
                                 x0=x0[r0:r0 + n])
                    done = self.done[r0:r0 + n]
                    for t in range(t0, t1):
                        smp = None if t == 0 else st.sample_args(
                            t - 1, r0, self.out[r0:r0 + n, t - 1], done, self.seed, self.Mx, self.mode, self.temp,
                            self.greedy, self.fix_pen)
                        st.step_fused(t, smp)
                    if t1 == N:
                        st.head()          # the last stroke: head + sampler
                        rc = lib.skr_mdn_sample_slabs(
                            st.ZS.data_ptr(), 128, st.S_o, n * 128, st._w["bo"].data_ptr(), n, self.Mx, self.mode,
                            self.temp, int(self.greedy), int(self.fix_pen), self.seed.data_ptr(), N - 1, r0,
                            self.out[r0, N - 1].data_ptr(), ld_out, st.X.data_ptr(), 5, done.data_ptr(),
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                        if rc != 0:
                            raise RuntimeError("skr_mdn_sample_slabs failed (%d)" % rc)
                continue
            with torch.cuda.stream(stream):
                if t0 == 0:
                    st.begin(zc[r0:r0 + n] if zc is not None else None, [s[r0:r0 + n] for s in state])
                    cy["x%d" % i] = x0[r0:r0 + n].contiguous()
                x = cy["x%d" % i]
                for t in range(t0, t1):
                    nx = torch.empty(n, 5, device=self.dev)

                    def sample(zs, ldz, nslab, slab, bias, r0=r0, n=n, t=t, nx=nx):
                        rc = lib.skr_mdn_sample_slabs(
                            zs.data_ptr(), ldz, nslab, slab, bias.data_ptr(), n, self.Mx, self.mode, self.temp,
                            int(self.greedy), int(self.fix_pen), self.seed.data_ptr(), t, r0,
                            self.out[r0, t].data_ptr(), ld_out, nx.data_ptr(), 5, self.done[r0:].data_ptr(),
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                        if rc != 0:
                            raise RuntimeError("skr_mdn_sample_slabs failed (%d)" % rc)
                    st.step(x, t, sample)
                    x = nx
                cy["x%d" % i] = x
        for _, _, _, stream in stp:
            if stream != main:
                main.wait_stream(stream)          # join

    @torch.no_grad()
    def _decode(self, t0: int, t1: int):
        """Decode steps [t0, t1); t0 == 0 starts a sketch (state, done flags)."""
        model, B = self.model, self.B
        if t0 == 0:
            self.done.zero_()
        stp = self._steppers()
        if stp is not None:
            fused = {st.fused for _, _, st, _ in stp}
            # fused step decoders draw stroke t inside step t + 1's launch: after
            # steps [t0, t1) the done flags cover strokes < t1 - 1
            self._lag = 1 if fused == {True} else (0 if fused == {False} else None)
            return self._decode_steppers(stp, t0, t1)
        self._lag = 0
        cy = self._carry
        if t0 == 0:
            cy["x"] = self.x0.clone()
            if self.kind == "vae":
                cfg = model.cfg
                lab = self.labels if cfg.num_classes > 0 else None
                cy["zc"] = model.condition(self.z if cfg.conditional else None, lab, B, self.dev)
                cy["state"] = model.initial_state(cy["zc"], B, self.dev)
            else:
                cy["zc"] = None
                cy["state"] = model.zero_state(B, self.dev)
        x, zc, state = cy["x"], cy["zc"], cy["state"]
        for t in range(t0, t1):
            if self.kind == "vae":
                zh, state = model.decode_step(x, zc, state)
            else:
                zh, state = model.step(x, state)
            nx = torch.empty(B, 5, device=self.dev)
            mdn_sample_device(zh.contiguous(), self.Mx, self.mode, self.temp, self.greedy, self.fix_pen, self.seed, t,
                              self.out[:, t], nx, self.done)
            x = nx
        cy["x"], cy["state"] = x, state

    def _exit_after(self, t1: int) -> bool:
        return self.early_exit and self._lag is not None and t1 < self.N and bool(self.done.all())

    def _pad_from(self, t: int):
        """Rows of steps [t, N) as the sampler emits them for finished rows."""
        if t < self.N:
            self.out[:, t:].zero_()
            self.out[:, t:, 4 if self.kind == "vae" else 3] = 1.0

    @torch.no_grad()
    def run(self, seed: int = 0, z: Optional[torch.Tensor] = None, labels: Optional[torch.Tensor] = None):
        if z is not None:
            self.z.copy_(z)
        elif self.kind == "vae":
            g = torch.Generator(device=self.dev).manual_seed(int(seed))
            self.z.copy_(torch.randn(self.z.shape, device=self.dev, generator=g))
        if labels is not None:
            self.labels.copy_(labels)
        self.seed.fill_(int(seed))
        ran = self.N
        if self.use_graph:
            # the graphs hold inference-cached weight copies (bf16): re-capture after a weight update
            from ..ops import gemm
            sig = (gemm.WEIGHTS_EPOCH[0],) + tuple(p._version for p in self.model.parameters())
            if self.graphs is not None and sig != self._sig:
                self.graphs = None
            self._sig = sig
            if self.graphs is None:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    for t0, t1 in self.ranges:
                        self._decode(t0, t1)
                torch.cuda.current_stream().wait_stream(s)
                self.graphs, pool = [], None
                for t0, t1 in self.ranges:
                    g = torch.cuda.CUDAGraph()
                    with capture(g, pool=pool):
                        self._decode(t0, t1)
                    pool = g.pool() if pool is None else pool
                    self.graphs.append(g)
            for (t0, t1), g in zip(self.ranges, self.graphs):
                g.replay()
                ran = t1
                if self._exit_after(t1):   # one host read per chunk
                    break
        else:
            for t0, t1 in self.ranges:
                self._decode(t0, t1)
                ran = t1
                if self._exit_after(t1):
                    break
        if ran < self.N:
            self._pad_from(ran - self._lag)   # strokes the skipped launches would have drawn: all padding
        self.steps_run = ran
        strokes = self.out.clone()
        stop_col = 4 if self.kind == "vae" else 3
        hits = strokes[:, :, stop_col] > 0
        lengths = torch.where(hits.any(1), hits.float().argmax(1) + 1, torch.full_like(hits[:, 0], self.N,
                                                                                      dtype=torch.long))
        if self.kind == "reference":
            strokes[:, :, 0:2] *= self.model.cfg.data_scale
        return strokes, lengths
