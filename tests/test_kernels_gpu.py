"""HIP kernels vs the fp32 PyTorch oracle (forward values and gradients).

Each test runs the same op twice on the GPU: once through the native
kernels (``ops.set_backend('hip')``) and once through the PyTorch oracle
(``'torch'``), with identical inputs, and compares outputs and input/weight
gradients. Dropout masks come from the shared stateless hash, so they match
exactly.
"""
import math

import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.models import cells as C
from sketch_rnn_amd.models.mdn import mdn_loss_torch
from sketch_rnn_amd.utils import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _restore():
    yield
    ops.set_backend("auto")
    ops.set_compute_dtype("fp32")
    from sketch_rnn_amd.ops.recurrent import check_cluster_errors
    torch.cuda.synchronize()
    check_cluster_errors(DEV)


def _run(backend, fn, inputs):
    ops.set_backend(backend)
    xs = [t.detach().clone().requires_grad_(t.requires_grad) for t in inputs]
    outs = fn(*xs)
    loss = sum((o * w).sum() for o, w in zip(outs, _weights(outs)))
    loss.backward()
    return [o.detach() for o in outs], [x.grad for x in xs]


_W = {}


def _weights(outs):
    key = tuple(tuple(o.shape) for o in outs)
    if key not in _W:
        g = torch.Generator(device=DEV).manual_seed(99)
        _W[key] = [torch.randn(o.shape, device=DEV, generator=g) for o in outs]
    return _W[key]


def _close(a, b, rtol, atol, what):
    for i, (x, y) in enumerate(zip(a, b)):
        if x is None and y is None:
            continue
        assert x is not None and y is not None, (what, i)
        err = (x - y).abs().max().item()
        ref = y.abs().max().item()
        assert err <= atol + rtol * ref, "%s[%d]: max err %.3e (ref max %.3e)" % (what, i, err, ref)


@pytest.mark.parametrize("H,ln,reset,keep", [(64, False, False, 1.0), (256, False, True, 1.0),
                                             (512, False, False, 0.9), (96, True, False, 1.0),
                                             (300, True, True, 0.85), (2048, True, False, 1.0),
                                             (600, True, True, 0.9), (1100, False, True, 0.8)])
def test_lstm_sequence_matches_oracle(H, ln, reset, keep):
    torch.manual_seed(0)
    T, B = 7, 5
    xp = torch.randn(T, B, 4 * H, device=DEV, requires_grad=True)
    W = (torch.randn(H, 4 * H, device=DEV) / math.sqrt(H)).requires_grad_()
    h0 = torch.randn(B, H, device=DEV, requires_grad=True) * 0.5
    c0 = torch.randn(B, H, device=DEV, requires_grad=True) * 0.5
    h0 = h0.detach().requires_grad_()
    c0 = c0.detach().requires_grad_()
    lnp = [torch.randn(4 * H, device=DEV).mul(0.1).add(1).requires_grad_(),
           torch.randn(4 * H, device=DEV).mul(0.1).requires_grad_(),
           torch.randn(H, device=DEV).mul(0.1).add(1).requires_grad_(),
           torch.randn(H, device=DEV).mul(0.1).requires_grad_()] if ln else []
    rst = (torch.rand(T, B, device=DEV) < 0.3).float() if reset else None
    seed = torch.tensor([17], device=DEV)

    def fn(xp, W, h0, c0, *lnp):
        lnt = tuple(lnp) if ln else None
        out, (hT, cT) = ops.lstm_sequence(xp, W, h0, c0, reset=rst, reset_h=h0 if reset else None,
                                          reset_c=c0 if reset else None, drop_keep=keep, drop_seed=seed,
                                          drop_stream=3, ln=lnt)
        return [out, hT, cT]

    inputs = [xp, W, h0, c0] + lnp
    o_h, g_h = _run("hip", fn, inputs)
    o_t, g_t = _run("torch", fn, inputs)
    _close(o_h, o_t, 1e-4, 1e-5, "out")
    _close(g_h, g_t, 1e-3, 1e-4, "grad")


@pytest.mark.parametrize("H,ln,keep", [(64, False, 1.0), (512, False, 0.9), (96, True, 0.8)])
def test_bilstm_sequence_matches_oracle(H, ln, keep):
    torch.manual_seed(5)
    T, B = 6, 4
    xs = [torch.randn(T, B, 4 * H, device=DEV, requires_grad=True) for _ in range(2)]
    Ws = [(torch.randn(H, 4 * H, device=DEV) / math.sqrt(H)).requires_grad_() for _ in range(2)]
    h0 = torch.zeros(B, H, device=DEV)
    lnp = []
    if ln:
        for _ in range(2):
            lnp += [torch.randn(4 * H, device=DEV).mul(0.1).add(1).requires_grad_(),
                    torch.randn(4 * H, device=DEV).mul(0.1).requires_grad_(),
                    torch.randn(H, device=DEV).mul(0.1).add(1).requires_grad_(),
                    torch.randn(H, device=DEV).mul(0.1).requires_grad_()]
    seed = torch.tensor([3], device=DEV)

    def fn(xf, xb, Wf, Wb, *lnp):
        lf, lb = (tuple(lnp[:4]), tuple(lnp[4:])) if ln else (None, None)
        of, ob = ops.bilstm_sequence(xf, xb, Wf, Wb, h0, h0, drop_keep=keep, drop_seed=seed, drop_stream=11,
                                     ln_f=lf, ln_b=lb)
        return [of, ob]

    inputs = xs + Ws + lnp
    o_h, g_h = _run("hip", fn, inputs)
    o_t, g_t = _run("torch", fn, inputs)
    _close(o_h, o_t, 1e-4, 1e-5, "out")
    _close(g_h, g_t, 1e-3, 1e-4, "grad")


@pytest.mark.parametrize("H,B,T,keep", [(512, 100, 9, 0.9), (256, 37, 6, 1.0), (2048, 64, 4, 0.9), (512, 128, 3, 0.8)])
def test_ln_lstm_chained_steps(H, B, T, keep):
    """ops.recurrent.LN_CHAIN (csrc/chain_step.hip skr_chain_ln_fwd / _bwd):
    the LayerNorm-LSTM cell rows of each step inside the launch of the
    product that feeds them, against the two-launch path and the fp32 oracle
    -- outputs, final states and every gradient, dropout on: error <= 1.5 x
    the two-launch error + 1e-3 of the largest element; NaN-poisoned slabs
    (a row reading ahead of its producer tiles) must not change a bit; the
    chained launches ran T times forward and T - 1 backward."""
    from sketch_rnn_amd.ops import recurrent
    torch.manual_seed(H + B)
    xp = torch.randn(T, B, 4 * H, device=DEV, requires_grad=True)
    W = (torch.randn(H, 4 * H, device=DEV) / math.sqrt(H)).requires_grad_()
    h0 = (torch.randn(B, H, device=DEV) * 0.5).requires_grad_()
    c0 = (torch.randn(B, H, device=DEV) * 0.5).requires_grad_()
    lnp = [torch.randn(4 * H, device=DEV).mul(0.1).add(1).requires_grad_(),
           torch.randn(4 * H, device=DEV).mul(0.1).requires_grad_(),
           torch.randn(H, device=DEV).mul(0.1).add(1).requires_grad_(),
           torch.randn(H, device=DEV).mul(0.1).requires_grad_()]
    seed = torch.tensor([23], device=DEV)

    def fn(xp, W, h0, c0, *lnp):
        out, (hT, cT) = ops.lstm_sequence(xp, W, h0, c0, drop_keep=keep, drop_seed=seed, drop_stream=5, ln=tuple(lnp))
        return [out, hT, cT]

    inputs = [xp, W, h0, c0] + lnp
    saved = recurrent.LN_CHAIN, recurrent.LN_CHAIN_POISON
    res = {}
    try:
        for name, backend, dt, chain, pois in (("ref", "torch", "fp32", False, False), ("plain", "hip", "bf16", False, False),
                                               ("chain", "hip", "bf16", True, False), ("chain_p", "hip", "bf16", True, True)):
            recurrent.LN_CHAIN, recurrent.LN_CHAIN_POISON = chain, pois
            ops.set_compute_dtype(dt)
            n0 = dict(recurrent.LN_CHAIN_STATS)
            o, g = _run(backend, fn, inputs)
            res[name] = o + g
            if chain:
                assert recurrent.LN_CHAIN_STATS["fwd"] - n0["fwd"] == T
                assert recurrent.LN_CHAIN_STATS["bwd"] - n0["bwd"] == T - 1
    finally:
        recurrent.LN_CHAIN, recurrent.LN_CHAIN_POISON = saved
        ops.set_compute_dtype("fp32")
    for i, (c, cp, p_, r) in enumerate(zip(res["chain"], res["chain_p"], res["plain"], res["ref"])):
        assert torch.isfinite(cp).all(), i
        assert torch.equal(c, cp), i
        scale = max(r.abs().max().item(), 1e-3)
        e_c = (c.float() - r).abs().max().item()
        e_p = (p_.float() - r).abs().max().item()
        assert e_c <= 1.5 * e_p + 1e-3 * scale, (i, e_c, e_p, scale)


@pytest.mark.parametrize("H,B,T,keep", [(512, 100, 9, 0.9), (256, 37, 6, 1.0), (1024, 64, 4, 0.9), (512, 128, 3, 0.8)])
def test_ln_lstm_skewed_forward(H, B, T, keep):
    """ops.recurrent.LN_SKEW (csrc/chain_step.hip skr_skew_ln_fwd): launch t
    runs the cell rows of step t and the h_t W_h tiles of step t + 1 (weight
    slice staged before the wait, h_t read with sc1 loads) -- against the
    chained steps and the fp32 oracle, outputs, final states and every
    gradient: error <= 1.5 x the chained error + 1e-3 of the largest
    element; NaN-poisoned h_t rows before every launch (a tile reading ahead
    of the rows) must not change a bit; T skewed launches per sequence."""
    from sketch_rnn_amd.ops import recurrent
    torch.manual_seed(H + B + 1)
    xp = torch.randn(T, B, 4 * H, device=DEV, requires_grad=True)
    W = (torch.randn(H, 4 * H, device=DEV) / math.sqrt(H)).requires_grad_()
    h0 = (torch.randn(B, H, device=DEV) * 0.5).requires_grad_()
    c0 = (torch.randn(B, H, device=DEV) * 0.5).requires_grad_()
    lnp = [torch.randn(4 * H, device=DEV).mul(0.1).add(1).requires_grad_(),
           torch.randn(4 * H, device=DEV).mul(0.1).requires_grad_(),
           torch.randn(H, device=DEV).mul(0.1).add(1).requires_grad_(),
           torch.randn(H, device=DEV).mul(0.1).requires_grad_()]
    seed = torch.tensor([29], device=DEV)

    def fn(xp, W, h0, c0, *lnp):
        out, (hT, cT) = ops.lstm_sequence(xp, W, h0, c0, drop_keep=keep, drop_seed=seed, drop_stream=5, ln=tuple(lnp))
        return [out, hT, cT]

    inputs = [xp, W, h0, c0] + lnp
    saved = recurrent.LN_CHAIN, recurrent.LN_SKEW, recurrent.LN_CHAIN_POISON
    res = {}
    try:
        for name, backend, dt, skew, pois in (("ref", "torch", "fp32", False, False), ("chain", "hip", "bf16", False, False),
                                              ("skew", "hip", "bf16", True, False), ("skew_p", "hip", "bf16", True, True)):
            recurrent.LN_CHAIN, recurrent.LN_SKEW, recurrent.LN_CHAIN_POISON = True, skew, pois
            ops.set_compute_dtype(dt)
            n0 = recurrent.LN_SKEW_STATS["fwd"]
            o, g = _run(backend, fn, inputs)
            res[name] = o + g
            if skew:
                assert recurrent.LN_SKEW_STATS["fwd"] - n0 == T
    finally:
        recurrent.LN_CHAIN, recurrent.LN_SKEW, recurrent.LN_CHAIN_POISON = saved
        ops.set_compute_dtype("fp32")
    for i, (c, k, kp, r) in enumerate(zip(res["chain"], res["skew"], res["skew_p"], res["ref"])):
        assert torch.isfinite(kp).all(), i
        assert torch.equal(k, kp), i
        scale = max(r.abs().max().item(), 1e-3)
        e_k = (k.float() - r).abs().max().item()
        e_c = (c.float() - r).abs().max().item()
        assert e_k <= 1.5 * e_c + 1e-3 * scale, (i, e_k, e_c, scale)


def test_lstm_sequence_bf16_close():
    torch.manual_seed(1)
    T, B, H = 9, 8, 512
    xp = torch.randn(T, B, 4 * H, device=DEV, requires_grad=True)
    W = (torch.randn(H, 4 * H, device=DEV) / math.sqrt(H)).requires_grad_()
    h0 = torch.zeros(B, H, device=DEV, requires_grad=True)
    c0 = torch.zeros(B, H, device=DEV, requires_grad=True)

    def fn(xp, W, h0, c0):
        out, (hT, cT) = ops.lstm_sequence(xp, W, h0, c0)
        return [out, hT, cT]

    ops.set_compute_dtype("bf16")
    o_h, g_h = _run("hip", fn, [xp, W, h0, c0])
    ops.set_compute_dtype("fp32")
    o_t, g_t = _run("torch", fn, [xp, W, h0, c0])
    _close(o_h, o_t, 3e-2, 3e-2, "out")
    _close(g_h, g_t, 5e-2, 5e-2, "grad")


@pytest.mark.parametrize("H,nd,B,reset,keep", [(512, 2, 100, False, 0.9), (256, 1, 37, True, 0.8),
                                               (512, 1, 70, True, 1.0), (256, 2, 5, False, 1.0)])
def test_fused_lstm_step_matches_unfused(H, nd, B, reset, keep):
    """csrc/lstm_fused.hip (GEMM + cell in one launch, bf16 operands) vs the
    split GEMM + cell path and the fp32 oracle."""
    from sketch_rnn_amd.ops import recurrent
    torch.manual_seed(2)
    T = 8
    xs = [torch.randn(T, B, 4 * H, device=DEV, requires_grad=True) for _ in range(nd)]
    Ws = [(torch.randn(H, 4 * H, device=DEV) / math.sqrt(H)).requires_grad_() for _ in range(nd)]
    h0 = (torch.randn(B, H, device=DEV) * 0.5).requires_grad_()
    c0 = (torch.randn(B, H, device=DEV) * 0.5).requires_grad_()
    rst = (torch.rand(T, B, device=DEV) < 0.3).float() if reset else None
    seed = torch.tensor([23], device=DEV)

    if nd == 1:
        def fn(xp, W, h0, c0):
            out, (hT, cT) = ops.lstm_sequence(xp, W, h0, c0, reset=rst, reset_h=h0 if reset else None,
                                              reset_c=c0 if reset else None, drop_keep=keep, drop_seed=seed,
                                              drop_stream=5)
            return [out, hT, cT]
        inputs = xs + Ws + [h0, c0]
    else:
        def fn(xf, xb, Wf, Wb):
            return list(ops.bilstm_sequence(xf, xb, Wf, Wb, torch.zeros(B, H, device=DEV),
                                            torch.zeros(B, H, device=DEV), drop_keep=keep, drop_seed=seed,
                                            drop_stream=11))
        inputs = xs + Ws
    saved = recurrent.FUSED_ENABLED
    try:
        ops.set_compute_dtype("bf16")
        recurrent.FUSED_ENABLED = True
        o_f, g_f = _run("hip", fn, inputs)
        recurrent.FUSED_ENABLED = False
        o_u, g_u = _run("hip", fn, inputs)
    finally:
        recurrent.FUSED_ENABLED = saved
    ops.set_compute_dtype("fp32")
    o_t, g_t = _run("torch", fn, inputs)
    _close(o_f, o_u, 1e-2, 1e-2, "fused vs unfused out")
    _close(g_f, g_u, 2e-2, 2e-2, "fused vs unfused grad")
    _close(o_f, o_t, 3e-2, 3e-2, "fused vs oracle out")
    _close(g_f, g_t, 5e-2, 5e-2, "fused vs oracle grad")


@pytest.mark.parametrize("H,Hh,E,keep", [(64, 32, 4, 1.0), (256, 64, 8, 0.9), (2048, 256, 32, 1.0)])
def test_hyper_sequence_matches_oracle(H, Hh, E, keep):
    torch.manual_seed(2)
    T, B, IN = 5, 4, 13
    p = C.HyperLSTMParams(IN, H, Hh, E).to(DEV)
    with torch.no_grad():  # move off the degenerate init so every path carries signal
        for prm in p.parameters():
            prm.add_(torch.randn_like(prm) * 0.05)
    names = [n for n, _ in p.named_parameters()]
    x = torch.randn(T, B, IN, device=DEV, requires_grad=True)
    st = [torch.randn(B, n, device=DEV).mul(0.3).requires_grad_() for n in (H, H, Hh, Hh)]
    seed = torch.tensor([5], device=DEV)

    def fn(x, h0, c0, hh0, hc0, *params):
        q = C.HyperLSTMParams.__new__(C.HyperLSTMParams)
        torch.nn.Module.__init__(q)
        q.in_size, q.hidden, q.hyper_units, q.embed, q.use_layer_norm = IN, H, Hh, E, True
        for n, v in zip(names, params):
            object.__setattr__(q, n, v)
        out, (hT, cT, hhT, hcT) = ops.hyper_sequence(q, x, h0, c0, hh0, hc0, drop_keep=keep, drop_seed=seed,
                                                     drop_stream=9)
        return [out, hT, cT, hhT, hcT]

    inputs = [x] + st + [v.detach().clone().requires_grad_() for v in p.parameters()]
    o_h, g_h = _run("hip", fn, inputs)
    o_t, g_t = _run("torch", fn, inputs)
    _close(o_h, o_t, 2e-4, 2e-5, "out")
    _close(g_h, g_t, 2e-3, 2e-4, "grad")


@pytest.mark.parametrize("dt,B,H,Hh,E", [("fp32", 4, 256, 64, 8), ("bf16", 100, 2048, 256, 32),
                                          ("bf16", 24, 512, 64, 8)])
def test_hyper_no_layernorm_vs_oracle(dt, B, H, Hh, E):
    """HyperLSTM with a plain main cell (use_layer_norm=False; the hyper cell
    stays a LayerNorm cell, models/cells.py hyper_lstm_step) on the HIP
    kernels against the fp32 oracle: fp32 operands tight, bf16 at bf16
    tolerances. The LayerNorm parameters do not exist on this path."""
    torch.manual_seed(3)
    T, IN = 5, 13
    p = C.HyperLSTMParams(IN, H, Hh, E, use_layer_norm=False).to(DEV)
    assert not hasattr(p, "ln_gamma")
    with torch.no_grad():
        for prm in p.parameters():
            prm.add_(torch.randn_like(prm) * 0.05)
    x = torch.randn(T, B, IN, device=DEV)
    st = [torch.randn(B, n, device=DEV) * 0.3 for n in (H, H, Hh, Hh)]
    w = torch.randn(T, B, H, device=DEV)
    res = []
    for backend, d in (("hip", dt), ("torch", "fp32")):
        ops.set_backend(backend)
        ops.set_compute_dtype(d)
        p.zero_grad()
        out, fin = ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=4, drop_stream=9, hyp_drop_keep=0.9)
        loss = (out * w).sum() + sum((f * (0.5 + 0.1 * k)).sum() for k, f in enumerate(fin))
        loss.backward()
        torch.cuda.synchronize()
        res.append([out.detach()] + [f.detach() for f in fin] + [q.grad.clone() for q in p.parameters()])
    ops.set_compute_dtype("fp32")
    if dt == "fp32":
        _close(res[0][:5], res[1][:5], 2e-4, 2e-5, "out")
        _close(res[0][5:], res[1][5:], 2e-3, 2e-4, "grad")
    else:
        _close(res[0][:1], res[1][:1], 3e-2, 3e-2, "out")
        _close(res[0][5:], res[1][5:], 6e-2, 6e-2, "grad")


def _hyper_setup(seed, T, B, IN, Z, H, Hh, E, jitter=0.05, state=0.0):
    torch.manual_seed(seed)
    p = C.HyperLSTMParams(IN + Z, H, Hh, E).to(DEV)
    with torch.no_grad():  # move off the degenerate init so every path carries signal
        for prm in p.parameters():
            prm.add_(torch.randn_like(prm) * jitter)
    x = torch.randn(T, B, IN, device=DEV)
    z = torch.randn(B, Z, device=DEV) if Z else None
    st = [torch.randn(B, n, device=DEV) * state for n in (H, H, Hh, Hh)]
    w = torch.randn(T, B, H, device=DEV)
    return p, x, z, st, w


def _hyper_run(p, x, z, st, w, keep=0.9, hkeep=1.0, fin_w=True):
    """One forward + backward of ops.hyper_sequence; returns [out, finals...,
    dz, parameter grads]."""
    p.zero_grad()
    zg = z.detach().clone().requires_grad_() if z is not None else None
    out, fin = ops.hyper_sequence(p, x, *st, drop_keep=keep, drop_seed=4, drop_stream=9, hyp_drop_keep=hkeep, zc=zg)
    loss = (out * w).sum()
    if fin_w:
        loss = loss + sum((f * (0.5 + 0.1 * k)).sum() for k, f in enumerate(fin))
    loss.backward()
    torch.cuda.synchronize()
    return [out.detach()] + [f.detach() for f in fin] + ([zg.grad] if zg is not None else []) + \
        [q.grad.clone() for q in p.parameters()]


def _names(p, z=True):
    return ["out", "h", "c", "hh", "hc"] + (["dz"] if z else []) + [n for n, _ in p.named_parameters()]


@pytest.mark.parametrize("H,Hh,E", [(512, 64, 8), (2048, 256, 32)])
def test_hyper_sequence_bf16_close(H, Hh, E):
    """bf16 HyperLSTM (grouped GEMMs, bf16 modulation vectors) against the
    fp32 oracle at bf16 tolerances."""
    p, x, z, st, w = _hyper_setup(12, 6, 100, 5, 16, H, Hh, E)
    res = []
    for backend, dt in (("hip", "bf16"), ("torch", "fp32")):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        res.append(_hyper_run(p, x, z, st, w, fin_w=False))
    _close(res[0][:1], res[1][:1], 3e-2, 3e-2, "out")
    _close(res[0][5:], res[1][5:], 6e-2, 6e-2, "grad")


@pytest.mark.parametrize("B,keep,hkeep", [(100, 0.9, 0.9), (37, 1.0, 1.0), (128, 0.9, 1.0), (192, 0.9, 1.0),
                                          (256, 1.0, 0.9)])
def test_hyper_mod_path_vs_oracle(B, keep, hkeep):
    """The fused modulation step (csrc/hyper_mod.hip: vec + gate
    pre-activations + LayerNorm partial sums; the main cell without its
    statistics exchange) is as close to the fp32 oracle as the plain chain
    (bf16-output modulation GEMM + in-launch exchange): per output / gradient,
    error(fused) <= 1.5 error(plain) + 1e-3 of the largest element."""
    from sketch_rnn_amd.ops import hyper as recurrent
    p, x, z, st, w = _hyper_setup(6, 7, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    runs = {}
    try:
        for name, backend, dt, fused in (("ref", "torch", "fp32", True), ("fused", "hip", "bf16", True),
                                         ("plain", "hip", "bf16", False)):
            recurrent.HYPER_MOD = fused
            ops.set_backend(backend)
            ops.set_compute_dtype(dt)
            runs[name] = _hyper_run(p, x, z, st, w, keep, hkeep)
    finally:
        recurrent.HYPER_MOD = True
    for i, n in enumerate(_names(p)):
        ref = runs["ref"][i].float()
        scale = max(ref.abs().max().item(), 1e-3)
        e_f = (runs["fused"][i].float() - ref).abs().max().item()
        e_p = (runs["plain"][i].float() - ref).abs().max().item()
        # (B > 128: the plain chain keeps fp32 modulation vectors -- the bf16-
        # output GEMM takes <= 128 rows -- so it is the stricter yardstick;
        # the fused path then has to stay within bf16 tolerance of the oracle)
        ok = e_f <= 1.5 * e_p + 1e-3 * scale or (B > 128 and e_f <= 3e-2 * scale)
        assert ok, (n, e_f, e_p, scale)


@pytest.mark.parametrize("H,Hh,E", [(2048, 256, 32), (512, 64, 8)])
def test_hyper_grouped_gemm_path_bitwise(H, Hh, E):
    """bf16 HyperLSTM with the grouped per-step GEMM launches equals the
    one-launch-per-product path bit for bit (same tiles, same sums)."""
    from sketch_rnn_amd.ops import gemm
    from sketch_rnn_amd.ops import hyper
    p, x, z, st, w = _hyper_setup(3, 4, 100, 13, 0, H, Hh, E, jitter=0.0)
    saved = gemm.GROUPED, hyper.CHAIN
    res = []
    try:
        ops.set_compute_dtype("bf16")
        ops.set_backend("hip")
        hyper.CHAIN = False   # (the chained launches: test_hyper_chained_launches_vs_unchained)
        for grouped in (True, False):
            gemm.GROUPED = grouped
            res.append(_hyper_run(p, x, z, st, w))
    finally:
        gemm.GROUPED, hyper.CHAIN = saved
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_hyper_long_sequence_vs_oracle():
    """T = 250 (the vae_large sequence length), H = 2048, the model's own
    initialisation. The recurrence is chaotic over 250 steps: a 1e-6 input
    perturbation of the fp32 oracle itself grows to ~0.1 in the outputs
    (scripts/long_seq_drift.py, profiles/r3/long_seq_drift.jsonl), so no fixed
    tolerance separates a kernel bug from rounding at t = 250. Checked
    instead: (1) the HIP fp32 path tracks the fp32 oracle -- outputs, dz and
    every weight gradient -- inside 4x the oracle's own sensitivity to that
    perturbation; (2) the bf16 path stays within 6 % over the first 20 steps
    (bf16 rounding ~1e-2 at t = 1, then the same exponential growth the
    perturbation shows: ~4e-2 at t = 20, saturated by t ~ 100)."""
    p, x, z, st, w = _hyper_setup(8, 250, 8, 5, 16, 2048, 256, 32, jitter=0.0)
    runs = {}
    for name, backend, dt, xx in (("ref", "torch", "fp32", x), ("pert", "torch", "fp32", x + 1e-6 * torch.randn_like(x)),
                                  ("hip32", "hip", "fp32", x), ("hip16", "hip", "bf16", x)):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        runs[name] = _hyper_run(p, xx, z, st, w, keep=1.0, fin_w=False)
    for i, n in enumerate(_names(p)):
        if n in ("h", "c", "hh", "hc"):
            continue
        ref = runs["ref"][i].float()
        scale = max(ref.abs().max().item(), 1e-3)
        e_h = (runs["hip32"][i].float() - ref).abs().max().item()
        e_p = (runs["pert"][i].float() - ref).abs().max().item()
        ok = e_h <= 4 * e_p + 1e-4 * scale
        assert ok, (n, e_h, e_p, scale)
    out16, out32 = runs["hip16"][0][:20].float(), runs["ref"][0][:20].float()
    err = (out16 - out32).abs().max().item()
    ok = err <= 6e-2 * out32.abs().max().item()
    assert ok, ("bf16 out, t < 20", err)


def _grad_cosines(runs, names, arm, ref="ref"):
    out = {}
    for i, n in enumerate(names):
        if n in ("out", "h", "c", "hh", "hc"):
            continue
        r, g = runs[ref][i].double().flatten(), runs[arm][i].double().flatten()
        if r.norm() == 0:
            continue
        out[n] = float(g @ r / (g.norm() * r.norm()))
    return out


def test_hyper_bf16_gradients_b100_t50_cosine():
    """Shipped numerics at the headline geometry: B = 100 rows (the fused
    forward / backward launches, the chained row-kernel backward), H = 2048,
    T = 50, the model's own initialisation, dropout on. Every weight gradient
    of the bf16 HIP path points the same way as the fp32 oracle's: cosine >=
    0.98 (measured 0.996-0.998; b_z >= 0.95: its gradient is a column sum of
    the bf16-stored dvec over all T*B rows that cancels to ~1e-2 of its
    terms' magnitude, so the storage rounding of the terms bounds it)."""
    p, x, z, st, w = _hyper_setup(21, 50, 100, 5, 16, 2048, 256, 32, jitter=0.0, state=0.0)
    runs = {}
    for name, backend, dt in (("ref", "torch", "fp32"), ("bf16", "hip", "bf16")):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        runs[name] = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9, fin_w=False)
    ops.set_compute_dtype("fp32")
    cos = _grad_cosines(runs, _names(p), "bf16")
    print("T=50 gradient cosines (bf16 HIP vs fp32 oracle):", cos)
    bad = [(n, c) for n, c in cos.items() if c < (0.95 if n == "b_z" else 0.98)]
    assert not bad, (bad, cos)


def test_hyper_t250_b100_gradients():
    """The full T = 250 at B = 100, H = 2048. With the model's own
    initialisation the recurrence is chaotic over 250 steps: bf16 rounding
    (~1e-2 per step) decorrelates the late trajectory from the fp32 one
    (measured gradient cosines ~0: no fixed tolerance separates a kernel bug
    from rounding there -- profiles/r3/long_seq_drift.jsonl). So, at the full
    geometry: (1) the HIP fp32 path tracks the fp32 oracle -- every weight
    gradient's cosine within 0.05 of the oracle's own cosine under a 1e-6
    input perturbation; (2) with contractive recurrent weights (W_h, hyp_W_h
    x 0.25: perturbations decay instead of growing) the bf16 path -- chained
    backward launches, bf16 modulation vectors, row kernels -- matches the
    oracle over all 250 steps: cosine >= 0.98 (b_z >= 0.95)."""
    p, x, z, st, w = _hyper_setup(21, 250, 100, 5, 16, 2048, 256, 32, jitter=0.0, state=0.0)
    runs = {}
    for name, backend, dt, xx in (("ref", "torch", "fp32", x), ("pert", "torch", "fp32", x + 1e-6 * torch.randn_like(x)),
                                  ("hip32", "hip", "fp32", x), ("bf16", "hip", "bf16", x)):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        runs[name] = _hyper_run(p, xx, z, st, w, keep=0.9, hkeep=0.9, fin_w=False)
    names = _names(p)
    c32, cp, c16 = (_grad_cosines(runs, names, a) for a in ("hip32", "pert", "bf16"))
    print("T=250 cosines: hip fp32", c32, "oracle perturbed", cp, "bf16 (chaotic)", c16)
    bad = [(n, c32[n], cp[n]) for n in c32 if c32[n] < cp[n] - 0.05]
    assert not bad, ("hip fp32 vs oracle", bad)
    with torch.no_grad():
        p.W_h.mul_(0.25)
        p.hyp_W_h.mul_(0.25)
    runs = {}
    for name, backend, dt in (("ref", "torch", "fp32"), ("bf16", "hip", "bf16")):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        runs[name] = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9, fin_w=False)
    ops.set_compute_dtype("fp32")
    c16 = _grad_cosines(runs, names, "bf16")
    print("T=250 contractive: bf16 cosines", c16)
    bad = [(n, c) for n, c in c16.items() if c < (0.95 if n == "b_z" else 0.98)]
    assert not bad, ("bf16 vs oracle, contractive", bad, c16)


@pytest.mark.parametrize("M,N,K,nd", [(100, 9216, 2304, 1), (100, 2304, 9216, 1), (100, 256, 24576, 1),
                                      (100, 24576, 256, 1), (7, 64, 64, 1), (128, 2048, 512, 2),
                                      (100, 512, 2048, 2), (256, 8192, 2048, 1), (512, 1024, 256, 1),
                                      (192, 8192, 2048, 1), (320, 1024, 2304, 1)])
def test_skinny_gemm_matches_torch(M, N, K, nd):
    """(M > 128 and not a multiple of 128: the grouped kernel's partial last row block.)"""
    from sketch_rnn_amd.ops import gemm
    torch.manual_seed(6)
    a = torch.randn(nd * M, K, device=DEV).to(torch.bfloat16)
    bt = torch.randn(nd, N, K, device=DEV).to(torch.bfloat16)
    S = gemm.plan_splits(M, N, K, nd)
    assert S >= 1
    out = torch.empty(S, nd * M, N, device=DEV)
    gemm.rec_gemm(a, bt if nd > 1 else bt[0], out, S, nd)
    ref = torch.bmm(a.float().view(nd, M, K), bt.float().transpose(1, 2)).reshape(nd * M, N)
    got = out.sum(0)
    err = (got - ref).abs().max().item()
    assert err <= 1e-3 * ref.abs().max().item() + 1e-3, (S, err)


@pytest.mark.parametrize("with_bias", [True, False])
def test_bilstm_input_proj_matches_torch(with_bias):
    """csrc/inproj.hip: both encoder directions' K=5 projections (reversed
    backward direction) and their weight / bias gradients."""
    from sketch_rnn_amd.ops.inproj import _BiInProj, bilstm_input_proj_torch
    torch.manual_seed(6)
    T, B, IN, G = 37, 13, 5, 768
    x = torch.randn(T, B, IN, device=DEV)
    lengths = torch.randint(1, T + 1, (B,), device=DEV)
    params = [torch.randn(IN, G, device=DEV, requires_grad=True) for _ in range(2)]
    params += [torch.randn(G, device=DEV, requires_grad=True) for _ in range(2)] if with_bias else [None, None]
    w = torch.randn(T, 2 * B, G, device=DEV)
    outs, grads = [], []
    for fn in (lambda *a: _BiInProj.apply(x, lengths, *a), lambda *a: bilstm_input_proj_torch(x, lengths, *a)):
        ps = [p.detach().clone().requires_grad_() if p is not None else None for p in params]
        y = fn(*ps)
        (y * w).sum().backward()
        outs.append(y.detach())
        grads.append([p.grad for p in ps if p is not None])
    _close([outs[0]], [outs[1]], 1e-5, 1e-5, "xp")
    _close(grads[0], grads[1], 1e-4, 1e-3, "grad")


@pytest.mark.parametrize("with_z,with_bias", [(True, True), (False, True), (True, False)])
def test_stroke_input_proj_matches_torch(with_z, with_bias):
    """csrc/inproj.hip bproj: [x | z broadcast] @ W + b with the z part once
    per sequence, and its W / bias / z gradients from one read of dxp."""
    from sketch_rnn_amd.ops.inproj import stroke_input_proj
    torch.manual_seed(8)
    T, B, IN, Z, G = 29, 11, 5, 16, 512
    x = torch.randn(T, B, IN, device=DEV)
    zc = torch.randn(B, Z, device=DEV, requires_grad=True) if with_z else None
    W = torch.randn(IN + (Z if with_z else 0), G, device=DEV, requires_grad=True)
    b = torch.randn(G, device=DEV, requires_grad=True) if with_bias else None
    w = torch.randn(T, B, G, device=DEV)
    res = []
    for backend in ("hip", "torch"):
        ops.set_backend(backend)
        ins = [t.detach().clone().requires_grad_() if t is not None else None for t in (zc, W, b)]
        y = stroke_input_proj(x, ins[0], ins[1], ins[2])
        (y * w).sum().backward()
        res.append([y.detach()] + [t.grad for t in ins if t is not None])
    _close(res[0][:1], res[1][:1], 1e-5, 1e-5, "xp")
    _close(res[0][1:], res[1][1:], 1e-4, 1e-3, "grad")


@pytest.mark.parametrize("T,B,G,dt,pad", [(250, 100, 8192, torch.bfloat16, 0), (37, 11, 1000, torch.bfloat16, 24),
                                          (29, 7, 2052, torch.float32, 0), (5, 3, 1001, torch.float32, 0)])
def test_bproj_reduce_wide_vs_narrow(T, B, G, dt, pad):
    """csrc/inproj.hip bproj_bwd_wide (16-byte loads, T split over 4 waves,
    wave-order LDS sum) against the narrow kernel and the fp32 oracle: S =
    sum_t dxp, P = sum_t x^T dxp per row, strided rows (pad) and partial
    column blocks included; G = 1001 takes the narrow kernel (no 16-byte
    alignment) under both settings."""
    from sketch_rnn_amd.ops import inproj
    torch.manual_seed(G)
    x = torch.randn(T, B, 5, device=DEV)
    buf = torch.randn(T, B, G + pad, device=DEV).to(dt)
    dxp = buf[..., :G]
    res = {}
    saved = inproj.BPROJ_WIDE
    try:
        for wide in (False, True):
            inproj.BPROJ_WIDE = wide
            res[wide] = inproj.bproj_reduce(x, dxp, raw=True)
    finally:
        inproj.BPROJ_WIDE = saved
    d = dxp.float()
    refS = d.sum(0)
    refP = torch.einsum("tbi,tbg->big", x, d)
    for S, P in res.values():
        assert (S - refS).abs().max().item() <= 1e-4 * refS.abs().max().item() + 1e-4
        assert (P - refP).abs().max().item() <= 1e-4 * refP.abs().max().item() + 1e-4
    if G % (8 if dt == torch.bfloat16 else 4):
        assert torch.equal(res[True][0], res[False][0]) and torch.equal(res[True][1], res[False][1])


def test_hyper_sequence_with_broadcast_z_matches_oracle():
    """HyperLSTM with a stroke-5 input + per-sequence z (bproj path) vs the
    oracle on the concatenated input."""
    torch.manual_seed(9)
    T, B, IX, Z, H, Hh, E = 6, 5, 5, 12, 256, 64, 8
    p = C.HyperLSTMParams(IX + Z, H, Hh, E).to(DEV)
    with torch.no_grad():
        for prm in p.parameters():
            prm.add_(torch.randn_like(prm) * 0.05)
    x = torch.randn(T, B, IX, device=DEV)
    zc = torch.randn(B, Z, device=DEV, requires_grad=True)
    st = [torch.randn(B, n, device=DEV).mul(0.3) for n in (H, H, Hh, Hh)]
    w = torch.randn(T, B, H, device=DEV)
    res = []
    for backend in ("hip", "torch"):
        ops.set_backend(backend)
        p.zero_grad()
        z = zc.detach().clone().requires_grad_()
        out, _ = ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=4, drop_stream=9, zc=z)
        (out * w).sum().backward()
        res.append([out.detach(), z.grad] + [q.grad.clone() for q in p.parameters()])
    _close(res[0][:1], res[1][:1], 2e-4, 2e-5, "out")
    _close(res[0][1:], res[1][1:], 2e-3, 2e-4, "grad")


def test_grouped_skinny_gemm_matches_torch():
    """Independent products in one grouped launch (csrc/skinny_gemm.hip)."""
    from sketch_rnn_amd.ops import gemm
    torch.manual_seed(4)
    shapes = [(100, 8192, 2048, 2), (100, 1024, 2304, 4), (37, 256, 24576, 32), (128, 512, 640, 1)]
    jobs, refs = [], []
    for M, N, K, S in shapes:
        a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
        bt = (torch.randn(N, K, device=DEV) / math.sqrt(K)).to(torch.bfloat16)
        out = torch.full((S, M, N), float("nan"), device=DEV)
        jobs.append((a, bt, out, S))
        refs.append(a.float() @ bt.float().t())
    gemm.rec_gemm_group(jobs)
    for (a, bt, out, S), ref in zip(jobs, refs):
        err = (out.sum(0) - ref).abs().max().item()
        assert err < 1e-3 * ref.abs().max().item() + 1e-3, (a.shape, bt.shape, S, err)


@pytest.mark.parametrize("mode,M", [("reference", 24), ("magenta", 20), ("magenta", 5)])
def test_mdn_loss_matches_oracle(mode, M):
    torch.manual_seed(3)
    N = 1000
    z = torch.randn(N, 3 + 6 * M, device=DEV)
    z[:, 3 + 3 * M:3 + 5 * M] *= 0.3
    z.requires_grad_()
    tgt = torch.zeros(N, 5, device=DEV)
    tgt[:, 0:2] = torch.randn(N, 2, device=DEV)
    tgt[torch.arange(N), 2 + torch.randint(0, 3, (N,))] = 1.0

    def fn(z):
        a = ops.mdn_loss(z, tgt, M, mode=mode)
        return list(a)

    o_h, g_h = _run("hip", fn, [z])
    ops.set_backend("torch")
    o_t, g_t = _run("torch", fn, [z])
    _close(o_h, o_t, 1e-5, 1e-5, "loss")
    _close(g_h, g_t, 1e-4, 1e-7, "dz")


def test_mdn_reference_clamp_zero_grad():
    M = 4
    z = torch.zeros(3, 3 + 6 * M, device=DEV)
    z[:, 3 + 3 * M:3 + 5 * M] = -8.0  # tiny sigmas
    tgt = torch.tensor([[50.0, 50.0, 0, 0, 1]] * 3, device=DEV)
    z.requires_grad_()
    ops.set_backend("hip")
    tot, shape, pen = ops.mdn_loss(z, tgt, M, mode="reference")
    assert abs(shape.item() - (-math.log(1e-20))) < 1e-3
    shape.backward()
    assert z.grad[:, 3:].abs().max().item() == 0.0


def test_fused_adam_matches_oracle():
    from sketch_rnn_amd.train.optim import FlatAdam
    torch.manual_seed(4)
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in [(37,), (5, 7), (300, 11)]]
    ps2 = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    for mode, clip in (("global_norm", 0.5), ("value", 0.01)):
        o1 = FlatAdam(ps, lr=0.01, eps=1e-3, clip_mode=mode, clip=clip)
        o2 = FlatAdam(ps2, lr=0.01, eps=1e-3, clip_mode=mode, clip=clip)
        for step in range(3):
            for a, b in zip(ps, ps2):
                g = torch.randn_like(a)
                a.grad.copy_(g)
                b.grad.copy_(g)
            ops.set_backend("hip")
            o1.step()
            ops.set_backend("torch")
            o2.step()
            torch.testing.assert_close(o1.flat, o2.flat, rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(o1.scalars[:2], o2.scalars[:2])


@pytest.mark.parametrize("kind,H,reset,dtype,xgrad", [("gru", 64, False, "fp32", True), ("gru", 256, True, "fp32", True),
                                                      ("gru", 300, True, "bf16", True), ("rnn", 256, True, "fp32", True),
                                                      ("rnn", 128, False, "bf16", True),
                                                      # data input (layer 0): csrc/inproj.hip projection + grads
                                                      ("gru", 256, True, "bf16", False),
                                                      ("rnn", 256, True, "bf16", False),
                                                      ("gru", 64, False, "fp32", False)])
def test_gru_rnn_sequence_matches_oracle(kind, H, reset, dtype, xgrad):
    torch.manual_seed(11)
    T, B, IN = 9, 6, 5
    Pcls = C.GRUParams if kind == "gru" else C.RNNParams
    p = Pcls(IN, H).to(DEV)
    x = torch.randn(T, B, IN, device=DEV, requires_grad=True)
    h0 = (torch.randn(B, H, device=DEV) * 0.5).requires_grad_()
    rst = (torch.rand(T, B, device=DEV) < 0.3).float() if reset else None

    def run(backend):
        ops.set_backend(backend)
        ops.set_compute_dtype(dtype if backend == "hip" else "fp32")
        xs = [x.detach().clone().requires_grad_(xgrad), h0.detach().clone().requires_grad_()]
        for q in p.parameters():
            q.grad = None
        out, hT = (ops.gru_sequence if kind == "gru" else ops.rnn_sequence)(p, xs[0], xs[1], reset=rst,
                                                                             reset_h=xs[1] if reset else None)
        w = _weights([out, hT])
        ((out * w[0]).sum() + (hT * w[1]).sum()).backward()
        gx = [xs[0].grad] if xgrad else []
        return [out.detach(), hT.detach()], gx + [xs[1].grad] + [q.grad.clone() for q in p.parameters()]

    o_h, g_h = run("hip")
    o_t, g_t = run("torch")
    tol = (3e-2, 3e-2) if dtype == "bf16" else (1e-4, 1e-4)
    _close(o_h, o_t, tol[0], tol[1], "out")
    _close(g_h, g_t, tol[0] * 10 if dtype == "bf16" else 1e-3, tol[1] * 10 if dtype == "bf16" else 1e-4, "grad")


@pytest.mark.parametrize("model", ["lstm", "gru", "rnn"])
def test_reference_model_train_step_hip(model):
    from sketch_rnn_amd.config import RefConfig
    from sketch_rnn_amd.data.loader import SketchLoader
    from sketch_rnn_amd.data.synthetic import synthetic_reference_corpus
    from sketch_rnn_amd.train.trainer import ReferenceTrainer, _to_device
    cfg = RefConfig(model=model, rnn_size=128, num_mixture=8, batch_size=16, seq_length=50)
    ld = SketchLoader(16, 50, 15.0, sketches=synthetic_reference_corpus(200, seed=0, max_len=60), seed=0)
    tr = ReferenceTrainer(cfg, ld, device=DEV, log=lambda s: None)
    costs = []
    for _ in range(4):
        x, y = ld.next_batch()
        costs.append(float(tr.train_step(_to_device(x, DEV), _to_device(y, DEV))["cost"]))
    assert all(math.isfinite(c) for c in costs), costs


def test_reference_model_bf16_grads_match_fp32():
    """Reference model in bf16 mode (layer-1 input projection and MDN head
    through bf16 MFMA GEMMs, head bias gradient by the column-sum kernel)
    against the same model in fp32: every parameter gradient within bf16
    tolerance."""
    from sketch_rnn_amd.config import RefConfig
    from sketch_rnn_amd.models.reference import SketchRNN
    cfg = RefConfig(rnn_size=256, num_mixture=24, batch_size=32, seq_length=60, keep_prob=1.0)
    m = SketchRNN(cfg, seed=3).to(DEV)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(32, 60, 5, generator=g) * 0.5
    y = torch.randn(32, 60, 5, generator=g) * 0.5
    pen = torch.randint(0, 3, (2, 32, 60), generator=g)
    for t, p in ((x, pen[0]), (y, pen[1])):
        t[..., 2:] = torch.nn.functional.one_hot(p, 3).float()
    x, y = x.to(DEV), y.to(DEV)
    grads = {}
    for dt in ("fp32", "bf16"):
        ops.set_backend("hip")
        ops.set_compute_dtype(dt)
        m.zero_grad(set_to_none=True)
        cost = m.loss(x, y, None, train=False)[0]
        cost.backward()
        grads[dt] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    for n, ref in grads["fp32"].items():
        got = grads["bf16"][n]
        rel = float((got - ref).norm() / ref.norm().clamp_min(1e-12))
        assert rel < 3e-2, (n, rel)


def test_colsum_many_equals_colsum():
    """skr_colsum_multi (several column reductions in one launch per pass, the
    HyperLSTM LayerNorm gamma / beta gradients) equals one colsum per pair
    bit for bit at the same row-slice counts for C >= 1024 (narrower ones
    split a slice over row groups: a different fixed order), and every
    result the fp32 oracle."""
    from sketch_rnn_amd.ops.reduce import colsum, colsum_many
    torch.manual_seed(3)
    R = 2500
    pairs = [(torch.randn(R, C, device=DEV).to(dt), torch.randn(R, C, device=DEV).to(dt) if wy else None)
             for C, dt, wy in ((8192, torch.bfloat16, True), (2048, torch.bfloat16, True), (256, torch.float32, True),
                               (1024, torch.bfloat16, False))]
    splits = [64, 128, 48, 100]
    got = colsum_many(pairs, splits)
    for (x, y), sp, (gxy, gx) in zip(pairs, splits, got):
        rxy, rx = colsum(x, y, sp)
        assert (gxy is None) == (y is None)
        if x.shape[1] >= 1024:
            assert torch.equal(gx, rx)
            if y is not None:
                assert torch.equal(gxy, rxy)
        refx = x.float().sum(0)
        assert (gx - refx).abs().max().item() <= 1e-3 * refx.abs().max().item() + 1e-3
        if y is not None:
            ref = (x.float() * y.float()).sum(0)
            assert (gxy - ref).abs().max().item() <= 1e-3 * ref.abs().max().item() + 1e-3
    dflt = colsum_many(pairs)       # default slices (narrow ones capped): close to the oracle
    for (x, y), (gxy, gx) in zip(pairs, dflt):
        ref = x.float().sum(0)
        assert (gx - ref).abs().max().item() <= 1e-3 * ref.abs().max().item() + 1e-3


def test_colsum_many_eight_columns_per_thread(monkeypatch):
    """skr_colsum_multi nc = 8 (every operand bf16: one 16-byte load per row
    and operand) against nc = 4 at the same row slices: bit for bit where
    both keep one row group per column (C >= 2048), and every result -- the
    narrow row-group layouts and a strided [T, nd, B, C] direction view
    included -- against the fp32 oracle, at explicit and default slices."""
    from sketch_rnn_amd.ops import reduce
    torch.manual_seed(4)
    bf = torch.bfloat16
    T, nd, B = 50, 2, 50
    enc = torch.randn(T, nd, B, 512, device=DEV).to(bf)
    ency = torch.randn(T, nd, B, 512, device=DEV).to(bf)
    pairs = [(torch.randn(2500, 8192, device=DEV).to(bf), torch.randn(2500, 8192, device=DEV).to(bf)),
             (torch.randn(2500, 2048, device=DEV).to(bf), None),
             (torch.randn(2500, 256, device=DEV).to(bf), torch.randn(2500, 256, device=DEV).to(bf)),
             (enc[:, 1], ency[:, 1])]
    for splits in ([64, 100, 48, 30], None):
        res = {}
        for nc in (4, 8):
            monkeypatch.setattr(reduce, "COLSUM_NC", nc)
            res[nc] = reduce.colsum_many(pairs, splits)
        for (x, y), (a_xy, a_x), (b_xy, b_x) in zip(pairs, res[4], res[8]):
            if splits is not None and x.shape[-1] >= 2048:
                assert torch.equal(a_x, b_x)
                if y is not None:
                    assert torch.equal(a_xy, b_xy)
            refx = x.float().sum((0, 1)) if x.dim() == 3 else x.float().sum(0)
            assert (b_x - refx).abs().max().item() <= 1e-3 * refx.abs().max().item() + 1e-3
            if y is not None:
                ref = (x.float() * y.float()).sum((0, 1)) if x.dim() == 3 else (x.float() * y.float()).sum(0)
                assert (b_xy - ref).abs().max().item() <= 1e-3 * ref.abs().max().item() + 1e-3


@pytest.mark.parametrize("shape,xdt,with_y", [((250, 100, 512), torch.float32, True), ((3, 7, 300), torch.bfloat16, False),
                                              ((250, 2, 100, 64), torch.float32, True),
                                              ((30000, 123), torch.float32, False)])   # the MDN head bias shape
def test_colsum_matches_torch(shape, xdt, with_y):
    from sketch_rnn_amd.ops.reduce import colsum
    torch.manual_seed(2)
    x = torch.randn(*shape, device=DEV).to(xdt)
    y = torch.randn(*shape, device=DEV) if with_y else None
    if len(shape) == 4:   # per-group reduction over a [T, nd, B, C] view
        xv, yv = x[:, 1], y[:, 1]
    else:
        xv, yv = x, y
    sxy, sx = colsum(xv, yv)
    dims = tuple(range(xv.dim() - 1))
    ref_x = xv.float().sum(dims)
    assert torch.allclose(sx, ref_x, rtol=1e-4, atol=1e-3)
    if with_y:
        assert torch.allclose(sxy, (xv.float() * yv).sum(dims), rtol=1e-4, atol=1e-3)


def test_inference_weight_cache_tracks_graph_training():
    """Inference paths cache low-precision weight copies; parameters updated by
    HIP-graph replays (no version bump) must invalidate them."""
    from sketch_rnn_amd.cli.vae_train import make_datasets
    from sketch_rnn_amd.config import VAEConfig
    from sketch_rnn_amd.train.trainer import VAETrainer
    cfg = VAEConfig(enc_rnn_size=64, dec_rnn_size=256, z_size=16, num_mixture=5, max_seq_len=40, batch_size=16,
                    dec_model="hyper", hyper_num_units=64, hyper_embedding_size=8, save_every=0)
    (tr_set, va, te), _ = make_datasets(cfg, None, 200)
    tr = VAETrainer(cfg, tr_set, va, te, device=DEV, save_dir="/tmp/skr_cache_test", log=lambda s: None,
                    compute_dtype="bf16", use_graph=True)
    e0 = tr.evaluate(te, max_batches=2)
    for _ in range(3):
        tr.train_step(*tr.batch_to_device(tr_set.random_batch()))
    e1 = tr.evaluate(te, max_batches=2)
    ops.set_backend("torch")
    try:
        e_ref = tr.evaluate(te, max_batches=2)   # oracle path: no caches at all
    finally:
        ops.set_backend("auto")
    assert e1["cost"] != e0["cost"]
    assert abs(e1["cost"] - e_ref["cost"]) < 0.05 * abs(e_ref["cost"]) + 0.02, (e1, e_ref)


@pytest.mark.parametrize("shape", [(2048, 8192), (2, 512, 2048), (133, 1000), (37, 61)])
def test_cast_transpose_matches_torch(shape):
    """csrc/convert.hip: both bf16 layouts bit-equal to torch's cast / transpose,
    including ragged edges and strided destinations."""
    from sketch_rnn_amd.ops import gemm
    torch.manual_seed(1)
    W = torch.randn(*shape, device=DEV)
    plain, trans = gemm.cast_transpose(W)
    torch.cuda.synchronize()
    assert torch.equal(plain, W.to(torch.bfloat16))
    assert torch.equal(trans, W.to(torch.bfloat16).transpose(-1, -2))
    if len(shape) == 2 and shape[1] % 4 == 0 and shape[0] % 4 == 0:
        R, C = shape
        big = torch.zeros(C, R + 64, dtype=torch.bfloat16, device=DEV)
        gemm.cast_transpose(W, trans=big[:, 64:], want_plain=False)
        torch.cuda.synchronize()
        assert torch.equal(big[:, 64:], W.to(torch.bfloat16).t())
        assert torch.count_nonzero(big[:, :64]) == 0


def test_hash_normal_kernel_matches_torch_emulation():
    """csrc/noise.hip (device-seed path of models.cells.hash_normal) against the
    int64 torch emulation of the same hash streams."""
    from sketch_rnn_amd.models import cells as C
    seed = torch.tensor([12345], dtype=torch.int64, device=DEV)
    k = C.hash_normal(seed, 0x5E, 3, (100, 128))
    t = C.hash_normal(12345, 0x5E, 3, (100, 128), device=DEV)
    torch.cuda.synchronize()
    assert torch.allclose(k, t, rtol=1e-5, atol=1e-5)
    assert abs(float(k.mean())) < 0.05 and abs(float(k.std()) - 1.0) < 0.05


@pytest.mark.parametrize("M,N,K,nd", [(100, 8192, 2048, 1), (37, 256, 24576, 1), (100, 2048, 512, 2), (256, 512, 1024, 1)])
def test_skinny_gemm_f32_matches_torch(M, N, K, nd):
    """fp32-operand skinny MFMA kernel (v_mfma_f32_16x16x4_f32) against an
    fp64 reference: the fp32 parity path of every recurrence."""
    from sketch_rnn_amd.ops import gemm
    torch.manual_seed(7)
    a = torch.randn(nd * M, K, device=DEV)
    bt = torch.randn(nd, N, K, device=DEV) / math.sqrt(K)
    S = gemm.plan_splits(M, N, K, nd, torch.float32)
    assert S >= 1
    out = torch.full((S, nd * M, N), float("nan"), device=DEV)
    gemm.rec_gemm(a, bt if nd > 1 else bt[0], out, S, nd)
    ref = torch.bmm(a.double().view(nd, M, K), bt.double().transpose(1, 2)).reshape(nd * M, N)
    got = out.sum(0).double()
    err = (got - ref).abs().max().item()
    assert err <= 1e-5 * ref.abs().max().item() + 1e-5, (S, err)


@pytest.mark.parametrize("n,K,M,N,cs,sliced", [(1, 25000, 2048, 8192, False, True), (1, 3001, 256, 2560, True, False),
                                               (2, 1000, 512, 512, False, False), (1, 777, 2304, 1024, True, True)])
@pytest.mark.parametrize("db", [0, 1, 2])
def test_wgrad_kernel_vs_fp32(n, K, M, N, cs, sliced, db):
    """Hand-written long-K weight-gradient GEMM (csrc/wgrad_gemm.hip) against
    an fp32 product of the same bf16 operands: headline shape (split-free),
    K tails (K % 32 != 0), batched directions, strided column-slice operands,
    split-K with the fused column sums; two launches bit-identical."""
    from sketch_rnn_amd.ops import gemm
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    torch.manual_seed(K)
    dev = torch.device("cuda")
    if sliced:   # a column slice of a wider saved buffer (the decoder's [h | hh] rows)
        a = torch.randn(n, K, M + 256, device=dev).to(torch.bfloat16)[:, :, :M]
    else:
        a = torch.randn(n, K, M, device=dev).to(torch.bfloat16)
    b = torch.randn(n, K, N, device=dev).to(torch.bfloat16)
    aa, bb = (a, b) if n > 1 else (a[0], b[0])
    assert gemm._wgrad_hip_ok(a, b)
    lib = native.require_hip().lib
    prev = lib.skr_wgrad_set_variant(-1)   # (returns the current fragment schedule)
    assert lib.skr_wgrad_set_variant(db) in (0, 1, 2)
    try:
        r1 = gemm.wgrad(aa, bb, colsum=cs)
        r2 = gemm.wgrad(aa, bb, colsum=cs)
    finally:
        lib.skr_wgrad_set_variant(prev)
    out1, cs1 = r1 if cs else (r1, None)
    out2, cs2 = r2 if cs else (r2, None)
    ref = torch.bmm(a.float().transpose(1, 2), b.float())
    if n == 1:
        ref = ref[0]
    scale = float(ref.abs().max())
    err = float((out1 - ref).abs().max())
    assert err <= 2e-5 * scale * math.sqrt(K / 1000) + 1e-4, (err, scale)
    assert torch.equal(out1, out2)
    if cs:
        cref = b[0].float().sum(0)
        cerr = float((cs1 - cref).abs().max())
        assert cerr <= 1e-4 * float(cref.abs().max()) + 1e-3, cerr
        assert torch.equal(cs1, cs2)


@pytest.mark.parametrize("M,ra", [(100, 3), (37, 4), (128, 6), (256, 3), (200, 3)])
def test_skinny_register_a_bitwise(M, ra):
    """ops.gemm.SKINNY_RA (csrc/glds_mma.h ra_mma: each wave's A fragments
    loaded straight into registers, only B through the LDS-DMA ring) against
    the LDS-staged kernel: the same fragments and k order, so bit-identical
    slabs for the plain launch (split-K, a column slice of a wider A like the
    HyperLSTM's [h | hh] rows) and the grouped launch (two problems, row
    blocks past 128, a partial last block)."""
    from sketch_rnn_amd.ops import gemm
    torch.manual_seed(M + ra)
    dev = torch.device("cuda")
    A = torch.randn(M, 2304, device=dev).to(torch.bfloat16)
    W1 = torch.randn(8192, 2048, device=dev).to(torch.bfloat16)     # B^T of h @ W_h
    W2 = torch.randn(1024, 2304, device=dev).to(torch.bfloat16)     # B^T of [h | hh] @ W_y
    saved = gemm.SKINNY_RA
    out = {}
    try:
        for v in (0, ra):
            gemm.SKINNY_RA = v
            o1 = torch.full((2, M, 8192), float("nan"), device=dev)
            o2 = torch.full((4, M, 1024), float("nan"), device=dev)
            if M <= 128:
                gemm.rec_gemm(A[:, :2048], W1, o1, 2)
                gemm.rec_gemm(A, W2, o2, 4)
            p1 = torch.full((2, M, 8192), float("nan"), device=dev)
            p2 = torch.full((4, M, 1024), float("nan"), device=dev)
            gemm.rec_gemm_group([(A[:, :2048], W1, p1, 2), (A, W2, p2, 4)])
            out[v] = (o1, o2, p1, p2)
    finally:
        gemm.SKINNY_RA = saved
    for k in range(4):
        if M > 128 and k < 2:
            continue
        assert torch.equal(out[0][k], out[ra][k]), k
    ref = A[:, :2048].float() @ W1.float().t()
    assert (out[ra][2].sum(0) - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()


@pytest.mark.parametrize("n,K,M,N,cs,sliced", [(1, 25000, 2048, 8192, False, True), (1, 3001, 256, 2560, True, False),
                                               (2, 1000, 512, 512, False, False), (1, 777, 2304, 1024, True, True),
                                               (1, 33, 256, 256, True, False)])
def test_wgrad_one_wave_kernel_bitwise(n, K, M, N, cs, sliced):
    """The one-wave-per-SIMD weight-gradient kernel (skr_wgrad_set_variant(2):
    4 waves of 128 x 128, fragments pipelined across the K-step) against the
    8-wave kernel (variant 1): the same fragments in the same k order per
    output element, so bit-identical products and column sums -- split-free,
    split-K, K tails (K = 33: one full and one 1-row K-step), batched,
    strided; and the bounded-grid accumulate form (background launches)."""
    from sketch_rnn_amd.ops import gemm
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    torch.manual_seed(K + 1)
    dev = torch.device("cuda")
    if sliced:
        a = torch.randn(n, K, M + 256, device=dev).to(torch.bfloat16)[:, :, :M]
    else:
        a = torch.randn(n, K, M, device=dev).to(torch.bfloat16)
    b = torch.randn(n, K, N, device=dev).to(torch.bfloat16)
    aa, bb = (a, b) if n > 1 else (a[0], b[0])
    lib = native.require_hip().lib
    prev = lib.skr_wgrad_set_variant(-1)
    res = {}
    try:
        for v in (1, 2):
            lib.skr_wgrad_set_variant(v)
            r = gemm.wgrad(aa, bb, colsum=cs)
            out, c = r if cs else (r, None)
            acc = out.clone()
            acc_cs = c.clone() if cs else None
            gemm.wgrad(aa, bb, colsum=cs, out=acc, cs_out=acc_cs, acc=True, max_grid=16)
            res[v] = (out, c, acc, acc_cs)
    finally:
        lib.skr_wgrad_set_variant(prev)
    for k in range(4):
        if res[1][k] is None:
            continue
        assert torch.equal(res[1][k], res[2][k]), k
    scale = float(res[2][0].abs().max())
    assert torch.allclose(res[2][2], 2 * res[2][0], rtol=1e-5, atol=1e-5 * scale)


@pytest.mark.parametrize("Hh,H,E", [(256, 2048, 32), (64, 256, 8)])
def test_hyper_fold_kernels_vs_torch(Hh, H, E):
    """csrc/hyper_fold.hip: P = W_z W_a per block in both bf16 layouts, q, qb,
    and the projection gradients, against the fp32 torch products (the
    headline shape, and E < 32 with its zero-padded LDS tile)."""
    from sketch_rnn_amd.ops import hyper
    from sketch_rnn_amd.utils import native
    torch.manual_seed(0)
    Wz = torch.randn(Hh, 12 * E, device=DEV) * 0.2
    bz = torch.randn(12 * E, device=DEV) * 0.2
    Wa = torch.randn(12, E, H, device=DEV) * 0.2
    bias = torch.randn(4 * H, device=DEV)
    lib = native.require_hip().lib
    Pl = torch.empty(Hh, 12 * H, dtype=torch.bfloat16, device=DEV)
    PlT = torch.empty(12 * H, Hh, dtype=torch.bfloat16, device=DEV)
    q = torch.empty(12, H, device=DEV)
    qb = torch.empty(12 * H, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    assert lib.skr_hyper_fold(Wz.data_ptr(), bz.data_ptr(), Wa.data_ptr(), bias.data_ptr(), Hh, H, E,
                              Pl.data_ptr(), PlT.data_ptr(), q.data_ptr(), qb.data_ptr(), st) == 0
    Pref = torch.bmm(Wz.view(Hh, 12, E).permute(1, 0, 2), Wa).permute(1, 0, 2).reshape(Hh, 12 * H)
    qref = torch.bmm(bz.view(12, 1, E), Wa).reshape(12, H)
    assert float((Pl.float() - Pref).abs().max()) <= 1e-2 * float(Pref.abs().max())
    assert torch.equal(PlT, Pl.t().contiguous())
    assert torch.allclose(q, qref, rtol=1e-5, atol=1e-5)
    qbr = qref.clone()
    qbr[8:] += bias.view(4, H)
    assert torch.allclose(qb, qbr.reshape(-1), rtol=1e-5, atol=1e-5)
    dP = torch.randn(Hh, 12 * H, device=DEV)
    sV = torch.randn(12 * H, device=DEV)

    class S:
        pass
    s = S()
    s.W_z, s.b_z, s.W_a = Wz, bz, Wa
    got = hyper._hyper_proj_grads(dP, sV, s, Hh, H, E)
    dPv = dP.view(Hh, 12, H).transpose(0, 1)
    Wz3 = Wz.view(Hh, 12, E).transpose(0, 1)
    ref = (torch.bmm(dPv, Wa.transpose(1, 2)).transpose(0, 1).reshape(Hh, 12 * E),
           torch.bmm(sV.view(12, 1, H), Wa.transpose(1, 2)).reshape(12 * E),
           torch.bmm(Wz3.transpose(1, 2), dPv) + bz.view(12, E, 1) * sV.view(12, 1, H),
           sV[8 * H:])
    for a, b in zip(got, ref):
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-3 * float(b.abs().max())), float((a - b).abs().max())


def test_small_gemm_group_equals_single_launches():
    """skr_small_gemm_group (several small products -- different shapes,
    strides, batch counts, split factors, bias / accumulate -- in one launch
    + one split-K sum launch) equals the one-launch-per-product results bit
    for bit (same tiles, same split-K order)."""
    from sketch_rnn_amd.ops import gemm
    torch.manual_seed(9)
    h, w1, w2 = torch.randn(100, 1024, device=DEV), torch.randn(1024, 128, device=DEV), torch.randn(1024, 128, device=DEV)
    b1 = torch.randn(128, device=DEV)
    z, d = torch.randn(100, 128, device=DEV), torch.randn(100, 4608, device=DEV)
    acc0 = torch.randn(100, 1024, device=DEV)
    A, Bm = torch.randn(12 * 32, device=DEV), torch.randn(12 * 512, device=DEV)
    ref = [gemm.small_mm(h, w1, b1), gemm.small_mm(h, w2), gemm.small_mm(z.t(), d),
           gemm.small_mm(d[:, :128], w1.t(), out=acc0.clone(), acc=True)]
    cb = torch.zeros(12, 32, 512, device=DEV)
    gemm.small_mm_batched(A, 0, 32, 1, 0, Bm, 0, 512, 0, 1, cb, 0, 32 * 512, 512, 32, 512, 1, 12)
    g = gemm.SmallGroup(DEV)
    got = [g.mm(h, w1, b1), g.mm(h, w2), g.mm(z.t(), d), g.mm(d[:, :128], w1.t(), out=acc0.clone(), acc=True)]
    cg = torch.zeros(12, 32, 512, device=DEV)
    g.batched(A, 0, 32, 1, 0, Bm, 0, 512, 0, 1, cg, 0, 32 * 512, 512, 32, 512, 1, 12)
    g.run()
    for a, b in zip(got + [cg], ref + [cb]):
        assert torch.equal(a, b)
    assert torch.allclose(ref[0], h @ w1 + b1, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("M,N,K,ta,tb,bias,acc", [(100, 128, 1024, False, False, True, False),
                                                  (100, 4608, 128, False, False, True, False),
                                                  (128, 4608, 100, True, False, False, False),
                                                  (100, 128, 8192, False, True, False, True),
                                                  (1024, 128, 100, True, False, False, False),
                                                  (37, 70, 45, True, True, True, True)])
def test_small_gemm_matches_torch(M, N, K, ta, tb, bias, acc):
    """csrc/small_gemm.hip (the latent / initial-state / z-projection
    products and their gradients): transposed views, bias, accumulate and
    split-K against the fp32 torch product."""
    from sketch_rnn_amd.ops import gemm
    torch.manual_seed(0)
    a = torch.randn(K, M, device=DEV).t() if ta else torch.randn(M, K, device=DEV)
    b = torch.randn(N, K, device=DEV).t() if tb else torch.randn(K, N, device=DEV)
    bv = torch.randn(N, device=DEV) if bias else None
    base = torch.randn(M, N, device=DEV)
    out = base.clone()
    gemm.small_mm(a, b, bv, out=out, acc=acc)
    ref = (a.double() @ b.double()) + (bv.double() if bias else 0) + (base.double() if acc else 0)
    err = (out.double() - ref).abs().max().item()
    assert err <= 1e-4 * max(ref.abs().max().item(), 1.0) * math.sqrt(K / 64), err


def test_hyper_backward_fused_cell_launch_bitwise(monkeypatch):
    """The backward order [main cell] -> [dvec P^T] -> [hyper cell + dR_main
    W_h^T in one launch] -> [dR_hyp W_y^T] (skr_skinny_gemm_group_cellbwd)
    equals the unfused order bit for bit at equal split counts, and stays as
    close to the fp32 oracle as the bf16 tolerance test requires."""
    from sketch_rnn_amd.ops import hyper
    monkeypatch.setitem(hyper.SPLITS, "sh", 64)   # dvec P^T at 64 splits in both orders
    p, x, z, st, w = _hyper_setup(4, 6, 100, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    ops.set_compute_dtype("bf16")
    ops.set_backend("hip")
    res = []
    saved = hyper.HYPER_BWD_FUSE, hyper.CHAIN
    try:
        hyper.CHAIN = False   # (the chained launches: test_hyper_chained_launches_vs_unchained)
        for fuse in (True, False):
            hyper.HYPER_BWD_FUSE = fuse
            res.append(_hyper_run(p, x, z, st, w))
    finally:
        hyper.HYPER_BWD_FUSE, hyper.CHAIN = saved
    for n, a, b in zip(_names(p), *res):
        assert torch.equal(a, b), n



@pytest.mark.parametrize("B,T,fin_w", [(100, 7, True), (100, 5, False), (37, 4, True), (128, 3, False), (192, 4, True),
                                       (256, 3, False)])
def test_hyper_chained_launches_vs_unchained(B, T, fin_w):
    """csrc/chain_step.hip: the main-cell backward rows inside the next step's
    dR_hyp W_y^T launch (an in-launch wait on an arrival counter, sc1 slab
    reads), against the unchained launches and the fp32 oracle --
    outputs, final states, dz and every weight gradient, dropout on, from a
    non-degenerate state (P != 0, h0 != 0). The row is the same source in
    another kernel (rounding-level differences from fp contraction), so:
    error(chained) <= 1.5 error(unchained) + 1e-3 of the largest element;
    and the chained path itself is run twice and must repeat bit for bit
    (the rotating counters carry over between calls)."""
    from sketch_rnn_amd.ops import hyper
    from sketch_rnn_amd.ops.recurrent import ROW_STATS
    p, x, z, st, w = _hyper_setup(4, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    runs, chained = {}, {}
    saved = hyper.CHAIN
    try:
        for name, backend, dt, chain in (("ref", "torch", "fp32", False), ("chain", "hip", "bf16", True),
                                         ("plain", "hip", "bf16", False), ("chain2", "hip", "bf16", True)):
            hyper.CHAIN = chain
            ops.set_backend(backend)
            ops.set_compute_dtype(dt)
            n0 = ROW_STATS["chain"]
            runs[name] = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9, fin_w=fin_w)
            chained[name] = ROW_STATS["chain"] - n0
    finally:
        hyper.CHAIN = saved
    # backward main cell: T - 1 chained launches (the last time step has no
    # W_y^T product before it)
    assert chained["chain"] == chained["chain2"] == T - 1 and chained["plain"] == 0, chained
    for i, n in enumerate(_names(p)):
        assert torch.equal(runs["chain"][i], runs["chain2"][i]), n
        ref = runs["ref"][i].float()
        scale = max(ref.abs().max().item(), 1e-3)
        e_c = (runs["chain"][i].float() - ref).abs().max().item()
        e_p = (runs["plain"][i].float() - ref).abs().max().item()
        assert e_c <= 1.5 * e_p + 1e-3 * scale, (n, e_c, e_p, scale)


@pytest.mark.parametrize("B,T,fin_w", [(100, 7, True), (100, 5, False), (37, 4, True), (128, 3, False), (192, 4, True)])
def test_hyper_forward_chain_vs_unchained(B, T, fin_w):
    """csrc/hyper_mod.hip skr_hyper_mod_chain: the main-cell rows of step t
    inside step t's modulation launch (every workgroup runs its modulation
    tile, arrives, then B * CHAIN_FWD_C of them run the main cell after an
    in-launch wait, g and the partial sums read with sc1 loads) against the
    two-launch path and the fp32 oracle -- outputs, final states, dz and every
    weight gradient, dropout on. Same arithmetic in another thread layout
    (row sums in another order), so error(chained) <= 1.5 error(two
    launches) + 1e-3 of the largest element; the chained path repeats bit for
    bit; it ran T times for B <= 128 and not at all above (two row blocks)."""
    from sketch_rnn_amd.ops import hyper
    p, x, z, st, w = _hyper_setup(5, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    runs, launched = {}, {}
    saved = hyper.CHAIN_FWD, hyper.CELL_MOD
    hyper.CELL_MOD = False   # (the plain arm: the hyper cell and modulation as two launches)
    try:
        for name, backend, dt, chain in (("ref", "torch", "fp32", False), ("chain", "hip", "bf16", True),
                                         ("plain", "hip", "bf16", False), ("chain2", "hip", "bf16", True)):
            hyper.CHAIN_FWD = chain
            ops.set_backend(backend)
            ops.set_compute_dtype(dt)
            n0 = hyper.CHAIN_FWD_STATS["launches"]
            runs[name] = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9, fin_w=fin_w)
            launched[name] = hyper.CHAIN_FWD_STATS["launches"] - n0
    finally:
        hyper.CHAIN_FWD, hyper.CELL_MOD = saved
    assert launched["chain"] == launched["chain2"] == (T if B <= 128 else 0) and launched["plain"] == 0, launched
    for i, n in enumerate(_names(p)):
        assert torch.equal(runs["chain"][i], runs["chain2"][i]), n
        ref = runs["ref"][i].float()
        scale = max(ref.abs().max().item(), 1e-3)
        e_c = (runs["chain"][i].float() - ref).abs().max().item()
        e_p = (runs["plain"][i].float() - ref).abs().max().item()
        assert e_c <= 1.5 * e_p + 1e-3 * scale, (n, e_c, e_p, scale)


@pytest.mark.parametrize("C,B", [(1, 100), (2, 100), (4, 64)])
def test_hyper_forward_chain_row_split(C, B):
    """The chained forward with one, two and four workgroups per main-cell row
    (ops.hyper.CHAIN_FWD_C) against the two-launch path: the first step's
    output -- no recurrence between them, only the row sums' order differs --
    within 1e-5 of the largest element; every output and gradient of the
    4-step sequence against the fp32 oracle as in
    test_hyper_forward_chain_vs_unchained (later steps see the first step's
    differences through bf16 roundings of h, amplified by the LayerNorms);
    and the chained launch ran every step (B C <= 256 workgroups: the
    launch's grid at H = 2048)."""
    from sketch_rnn_amd.ops import hyper
    T = 4
    p, x, z, st, w = _hyper_setup(6, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    saved = hyper.CHAIN_FWD, hyper.CHAIN_FWD_C, hyper.CELL_MOD
    hyper.CELL_MOD = False   # (the plain arm: the hyper cell and modulation as two launches)
    runs = {}
    try:
        for name, backend, dt, chain in (("ref", "torch", "fp32", False), ("plain", "hip", "bf16", False),
                                         ("chain", "hip", "bf16", True)):
            hyper.CHAIN_FWD, hyper.CHAIN_FWD_C = chain, C
            ops.set_backend(backend)
            ops.set_compute_dtype(dt)
            n0 = hyper.CHAIN_FWD_STATS["launches"]
            runs[name] = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9)
            assert hyper.CHAIN_FWD_STATS["launches"] - n0 == (T if chain else 0)
    finally:
        hyper.CHAIN_FWD, hyper.CHAIN_FWD_C, hyper.CELL_MOD = saved
    o_p, o_c = runs["plain"][0][0], runs["chain"][0][0]
    assert (o_p - o_c).abs().max().item() <= 1e-5 * o_p.abs().max().item()
    for i, n in enumerate(_names(p)):
        ref = runs["ref"][i].float()
        scale = max(ref.abs().max().item(), 1e-3)
        e_c = (runs["chain"][i].float() - ref).abs().max().item()
        e_p = (runs["plain"][i].float() - ref).abs().max().item()
        assert e_c <= 1.5 * e_p + 1e-3 * scale, (n, e_c, e_p, scale)


@pytest.mark.parametrize("B,T", [(100, 6), (128, 3), (65, 4), (37, 3)])
def test_hyper_cell_and_modulation_one_launch(B, T):
    """csrc/hyper_mod.hip skr_hyper_cell_mod: wave 0 of modulation workgroup b
    runs the hyper cell of row b (row kernel body, hh stored write-through),
    every tile prefetches P / xh / R, waits for all rows and reads hh with sc1
    loads -- against the two launches and the fp32 oracle (outputs, finals,
    dz, every gradient; dropout on): error <= 1.5 x the two-launch error +
    1e-3 of the largest element (the row body sums in another order than the
    clustered hyper cell); NaN-poisoned hh rows before every launch (a tile
    reading ahead of the rows) must not change a bit; it ran T times for
    65 <= B <= 128 and not at all outside."""
    from sketch_rnn_amd.ops import hyper
    p, x, z, st, w = _hyper_setup(7, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    runs, launched = {}, {}
    saved = hyper.CELL_MOD, hyper.CELL_MOD_POISON
    try:
        for name, backend, dt, on, pois in (("ref", "torch", "fp32", False, False), ("cm", "hip", "bf16", True, False),
                                            ("plain", "hip", "bf16", False, False), ("cm_p", "hip", "bf16", True, True)):
            hyper.CELL_MOD, hyper.CELL_MOD_POISON = on, pois
            ops.set_backend(backend)
            ops.set_compute_dtype(dt)
            n0 = hyper.CELL_MOD_STATS["launches"]
            runs[name] = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9)
            launched[name] = hyper.CELL_MOD_STATS["launches"] - n0
    finally:
        hyper.CELL_MOD, hyper.CELL_MOD_POISON = saved
    want = T if 65 <= B <= 128 else 0
    assert launched["cm"] == launched["cm_p"] == want and launched["plain"] == 0, launched
    for i, n in enumerate(_names(p)):
        assert torch.isfinite(runs["cm_p"][i]).all(), n
        assert torch.equal(runs["cm"][i], runs["cm_p"][i]), n
        ref = runs["ref"][i].float()
        scale = max(ref.abs().max().item(), 1e-3)
        e_c = (runs["cm"][i].float() - ref).abs().max().item()
        e_p = (runs["plain"][i].float() - ref).abs().max().item()
        assert e_c <= 1.5 * e_p + 1e-3 * scale, (n, e_c, e_p, scale)


@pytest.mark.parametrize("B,T,fin_w", [(100, 7, True), (100, 5, False), (37, 4, True), (128, 3, False),
                                       (192, 4, True), (256, 3, False)])
def test_hyper_three_stage_chain_bitwise(B, T, fin_w):
    """csrc/chain_step.hip skr_chain_bwd_main3: dvec P^T computed by the
    producer workgroups of the chained launch (weight slice staged in LDS
    while the rows compute, A operand through sc1 loads after the rows'
    counter) equals the separate dvec P^T launch bit for bit -- the same
    fragments, k order and MFMA -- for every output and gradient; and the
    launch really ran T - 1 times (B <= 128).  At 4 dR_hyp W_y^T slabs: the
    default cap of 2 leaves fewer producer tiles than dvec P^T tail tiles, so
    the three-stage launch declines (-2) and the two-stage chain runs."""
    from sketch_rnn_amd.ops import hyper
    from sketch_rnn_amd.ops.recurrent import ROW_STATS
    p, x, z, st, w = _hyper_setup(8, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    saved = hyper.CHAIN, hyper.CHAIN3, hyper.SAY_CAP
    runs = {}
    try:
        hyper.CHAIN, hyper.SAY_CAP = True, 4
        for c3 in (True, False, True):
            hyper.CHAIN3 = c3
            n0 = ROW_STATS["chain3"]
            runs.setdefault(c3, []).append(_hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9, fin_w=fin_w))
            # (B > 128: the tail is one 128-row block only -- not taken, two-stage chain)
            assert ROW_STATS["chain3"] - n0 == ((T - 1) if (c3 and B <= 128) else 0)
    finally:
        hyper.CHAIN, hyper.CHAIN3, hyper.SAY_CAP = saved
    for n, a, b, c in zip(_names(p), runs[True][0], runs[False][0], runs[True][1]):
        assert torch.equal(a, c), n
        assert torch.equal(a, b), n


@pytest.mark.parametrize("B,T", [(100, 7), (37, 4), (128, 3), (192, 4)])
def test_hyper_chained_rows_split_over_two_workgroups(B, T):
    """ops.hyper.CHAIN_CL = 2: each chained main-cell backward row on two
    workgroups (waves 4-7 of each end at once; the LayerNorm-backward row
    sums exchanged in-launch) against one workgroup per row and the fp32
    oracle: error <= 1.5 x the one-workgroup error + 1e-3 of the largest
    element for every output and gradient, NaN-poisoned slabs never read
    early, and bit-identical repeats."""
    from sketch_rnn_amd.ops import hyper
    from sketch_rnn_amd.ops.recurrent import ROW_STATS
    p, x, z, st, w = _hyper_setup(11, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    saved = hyper.CHAIN, hyper.CHAIN_CL, hyper.CHAIN_POISON
    runs = {}
    try:
        hyper.CHAIN = True
        for name, backend, dt, cl, pois in (("ref", "torch", "fp32", 1, False), ("one", "hip", "bf16", 1, False),
                                            ("two", "hip", "bf16", 2, False), ("two_p", "hip", "bf16", 2, True)):
            hyper.CHAIN_CL, hyper.CHAIN_POISON = cl, pois
            ops.set_backend(backend)
            ops.set_compute_dtype(dt)
            n0 = ROW_STATS["chain"]
            runs[name] = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9)
            if backend == "hip":
                assert ROW_STATS["chain"] - n0 == T - 1
    finally:
        hyper.CHAIN, hyper.CHAIN_CL, hyper.CHAIN_POISON = saved
    for i, n in enumerate(_names(p)):
        assert torch.equal(runs["two"][i], runs["two_p"][i]), n
        ref = runs["ref"][i].float()
        scale = max(ref.abs().max().item(), 1e-3)
        e_2 = (runs["two"][i].float() - ref).abs().max().item()
        e_1 = (runs["one"][i].float() - ref).abs().max().item()
        assert e_2 <= 1.5 * e_1 + 1e-3 * scale, (n, e_2, e_1, scale)


@pytest.mark.parametrize("B,T", [(100, 7), (192, 4)])
def test_hyper_chained_rows_never_overtake_the_counter(B, T):
    """Poison mode (ops.hyper.CHAIN_POISON): the d[h | hh] slabs (and, for the
    three-stage launch, the dvec rows) are NaN-filled before every chained
    launch, so a main-cell row that read them before its producer tiles had
    written them -- or a dvec P^T tile that read dvec before the rows had --
    would carry NaN into the gradients. The forward chain (ops.hyper.CHAIN_FWD,
    switched on here) is poisoned the same way: g and its partial sums are
    NaN-filled before every chained modulation launch. Every output and
    gradient must be finite and equal to the unpoisoned chained run bit for bit."""
    from sketch_rnn_amd.ops import hyper
    p, x, z, st, w = _hyper_setup(5, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    saved = hyper.CHAIN, hyper.CHAIN_POISON, hyper.CHAIN_FWD
    try:
        hyper.CHAIN = hyper.CHAIN_FWD = True
        hyper.CHAIN_POISON = False
        clean = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9)
        hyper.CHAIN_POISON = True
        pois = _hyper_run(p, x, z, st, w, keep=0.9, hkeep=0.9)
    finally:
        hyper.CHAIN, hyper.CHAIN_POISON, hyper.CHAIN_FWD = saved
    for n, a, b in zip(_names(p), clean, pois):
        assert torch.isfinite(b).all(), n
        assert torch.equal(a, b), n


def test_hyper_background_weight_grads_vs_serial():
    """ops.hyper.BG_WGRAD: dW_h, dW_y and dP (+ its column sums) computed in
    T-chunks on a side stream while the backward scan runs, with bounded
    grids and in-place accumulation, against the same products after the
    scan: equal up to fp32 summation order (the chunk partial sums are added
    in a different association), bit-identical outputs and non-weight
    gradients, and bit-identical repeats (fixed chunk order)."""
    from sketch_rnn_amd.ops import hyper
    T, B = 64, 100
    p, x, z, st, w = _hyper_setup(9, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    saved = hyper.BG_WGRAD, hyper.BG_CHUNK, hyper.BG_GRID
    try:
        hyper.BG_CHUNK, hyper.BG_GRID = 20, 16   # chunks [44, 64) [24, 44) [4, 24) on the side stream, [0, 4) last
        hyper.BG_WGRAD = False
        ser = _hyper_run(p, x, z, st, w)
        hyper.BG_WGRAD = True
        bg1 = _hyper_run(p, x, z, st, w)
        bg2 = _hyper_run(p, x, z, st, w)
    finally:
        hyper.BG_WGRAD, hyper.BG_CHUNK, hyper.BG_GRID = saved
    names = _names(p)
    chunked = {"W_h", "hyp_W_h", "hyp_W_x", "W_z", "b_z", "W_a", "bias"}
    for n, a, b, c in zip(names, ser, bg1, bg2):
        assert torch.equal(b, c), n
        if n in chunked:
            scale = max(a.abs().max().item(), 1e-6)
            assert (a - b).abs().max().item() <= 1e-5 * scale, (n, (a - b).abs().max().item(), scale)
        else:
            assert torch.equal(a, b), n

