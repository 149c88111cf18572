"""Model math on CPU (fp32/fp64 oracles): MDN head (R10-R12) vs the literal
probability-space transcription, clamp semantics, gradcheck; the stateless
dropout hash; recurrences with the eoc reset (R8); reference model variants
(R7); VAE (N1-N7) loss terms, state layouts and conditioning."""
import math

import numpy as np
import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.config import RefConfig, VAEConfig
from sketch_rnn_amd.models import cells as C
from sketch_rnn_amd.models.mdn import mdn_loss_prob_space, mdn_loss_torch, mixture_coef
from sketch_rnn_amd.models.reference import SketchRNN
from sketch_rnn_amd.models.vae import SketchVAE, reverse_padded
from sketch_rnn_amd.ops.recurrent_torch import lstm_sequence_torch


def _mdn_inputs(N=64, M=5, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    z = torch.randn(N, 3 + 6 * M, generator=g, dtype=torch.float64) * scale
    t = torch.zeros(N, 5, dtype=torch.float64)
    t[:, :2] = torch.randn(N, 2, generator=g, dtype=torch.float64)
    t[torch.arange(N), 2 + torch.randint(0, 3, (N,), generator=g)] = 1.0
    return z, t


def test_mdn_reference_matches_prob_space():
    z, t = _mdn_inputs()
    a = mdn_loss_torch(z, t, 5, mode="reference")
    b = mdn_loss_prob_space(z, t, 5)
    for x, y in zip(a, b):
        assert abs(float(x) - float(y)) < 1e-5 * max(1.0, abs(float(y)))


def test_mdn_clamp_value_and_zero_grad():
    z, t = _mdn_inputs(N=8)
    t[:4, :2] = 1e3  # far from every component: S << 1e-20
    z = z.clone().requires_grad_()
    tot, shape, pen = mdn_loss_torch(z, t, 5, mode="reference")
    ref = mdn_loss_prob_space(z.detach(), t, 5)
    assert abs(float(shape) - float(ref[1])) < 1e-6 * float(ref[1])
    shape.backward()
    assert torch.all(z.grad[:4] == 0)          # clamped rows: gradient goes to the constant
    assert torch.any(z.grad[4:] != 0)


def test_mdn_gradcheck_both_modes():
    z, t = _mdn_inputs(N=6, M=3)
    z.requires_grad_()
    for mode in ("reference", "magenta"):
        assert torch.autograd.gradcheck(lambda zz: mdn_loss_torch(zz, t, 3, mode=mode)[0], (z,), eps=1e-6, atol=1e-5)


def test_mdn_magenta_mask_and_eval_weighting():
    z, t = _mdn_inputs(N=10, M=4)
    t[5:, 2:] = torch.tensor([0.0, 0.0, 1.0], dtype=torch.float64)  # padding (p3)
    tot, shape, pen = mdn_loss_torch(z, t, 4, mode="magenta", is_training=True)
    pi, mu1, mu2, s1, s2, rho, _, pl = mixture_coef(z, 4)
    dx, dy = t[:, 0:1] - mu1, t[:, 1:2] - mu2
    zz = (dx / s1) ** 2 + (dy / s2) ** 2 - 2 * rho * dx * dy / (s1 * s2)
    pdf = torch.exp(-zz / (2 * (1 - rho ** 2))) / (2 * math.pi * s1 * s2 * torch.sqrt(1 - rho ** 2))
    fs = 1 - t[:, 4]
    ls = -torch.log((pi * pdf).sum(1) + 1e-6) * fs
    ce = -(t[:, 2:] * torch.log_softmax(pl, -1)).sum(1)
    assert abs(float(shape) - float(ls.mean())) < 1e-9
    assert abs(float(pen) - float(ce.mean())) < 1e-9
    _, _, pen_eval = mdn_loss_torch(z, t, 4, mode="magenta", is_training=False)
    assert abs(float(pen_eval) - float((ce * fs).mean())) < 1e-9


def test_hash_uniform_deterministic_and_uniform():
    a = C.hash_uniform(5, 3, 7, (1000, 10))
    b = C.hash_uniform(torch.tensor([5]), 3, 7, (1000, 10))
    assert torch.equal(a, b)
    assert not torch.equal(a, C.hash_uniform(5, 3, 8, (1000, 10)))
    assert not torch.equal(a, C.hash_uniform(5, 4, 7, (1000, 10)))
    assert 0.0 <= float(a.min()) and float(a.max()) < 1.0
    assert abs(float(a.mean()) - 0.5) < 0.01
    m = C.dropout_mask(1, 2, 3, (400, 100), 0.8)
    assert abs(float((m > 0).float().mean()) - 0.8) < 0.01 and abs(float(m.max()) - 1.25) < 1e-6


def test_lstm_reset_semantics():
    torch.manual_seed(0)
    T, B, H = 6, 3, 8
    xp = torch.randn(T, B, 4 * H)
    W = torch.randn(H, 4 * H) * 0.3
    h0, c0 = torch.randn(B, H), torch.randn(B, H)
    reset = torch.zeros(T, B)
    reset[2, 1] = 1.0
    out, _ = lstm_sequence_torch(xp, W, h0, c0, reset=reset, reset_h=h0, reset_c=c0)
    # row 1 after the reset == a fresh run from (h0, c0) starting at t=3
    fresh, _ = lstm_sequence_torch(xp[3:, 1:2], W, h0[1:2], c0[1:2])
    assert torch.allclose(out[3:, 1:2], fresh, atol=1e-6)
    plain, _ = lstm_sequence_torch(xp, W, h0, c0)
    assert torch.allclose(out[:, 0], plain[:, 0]) and torch.allclose(out[:3], plain[:3])


def test_lstm_pointwise_formula():
    g = torch.randn(4, 4 * 5)
    c = torch.randn(4, 5)
    h, c2 = C.lstm_pointwise(g, c, 1.0)
    i, j, f, o = g.split(5, -1)
    ce = c * torch.sigmoid(f + 1.0) + torch.sigmoid(i) * torch.tanh(j)
    assert torch.allclose(c2, ce, atol=1e-6) and torch.allclose(h, torch.tanh(ce) * torch.sigmoid(o), atol=1e-6)


@pytest.mark.parametrize("model,layers", [("lstm", 2), ("lstm", 1), ("lstm", 3), ("gru", 2), ("rnn", 2)])
def test_reference_model_variants(model, layers):
    cfg = RefConfig(rnn_size=16, num_layers=layers, model=model, num_mixture=3, keep_prob=0.8)
    m = SketchRNN(cfg, seed=0)
    B, T = 4, 9
    x = torch.zeros(B, T, 5)
    x[:, :, :2] = torch.randn(B, T, 2)
    x[:, :, 4] = 1
    x[:, 4, 3], x[:, 4, 4] = 1, 0
    y = torch.roll(x, -1, 1)
    cost, shape, pen, final = m.loss(x, y, None, train=True, drop_seed=3)
    cost.backward()
    assert torch.isfinite(cost) and len(final) == layers
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters())


def test_reference_model_eoc_reset_to_batch_initial_state():
    cfg = RefConfig(rnn_size=16, num_mixture=3, keep_prob=1.0)
    m = SketchRNN(cfg, seed=1)
    B, T = 2, 8
    x = torch.randn(B, T, 5)
    x[:, :, 2:] = 0
    x[:, :, 4] = 1
    x[0, 3, 3], x[0, 3, 4] = 1, 0
    st = [(torch.randn(B, 16), torch.randn(B, 16)) for _ in range(2)]
    z, _ = m.forward(x, st, train=False)
    z = z.view(T, B, -1)
    st0 = [(h[0:1], c[0:1]) for h, c in st]
    z2, _ = m.forward(x[0:1, 4:], st0, train=False)
    assert torch.allclose(z[4:, 0], z2.view(T - 4, -1), atol=1e-5)


def test_reverse_padded():
    x = torch.arange(2 * 5).view(5, 2, 1).float()   # [T, B, 1]
    r = reverse_padded(x, torch.tensor([3, 5]))
    assert r[:, 0, 0].tolist() == [4, 2, 0, 6, 8]
    assert r[:, 1, 0].tolist() == [9, 7, 5, 3, 1]


def _vae_batch(cfg, B=4, seed=0):
    from sketch_rnn_amd.data.dataset import StrokeDataset
    from sketch_rnn_amd.data.synthetic import synthetic_corpus
    s, l = synthetic_corpus(16, seed=seed, max_len=cfg.max_seq_len, n_classes=max(cfg.num_classes, 1))
    ds = StrokeDataset(s, B, cfg.max_seq_len, labels=l)
    ds.normalize()
    x, lens, lab = ds.random_batch()
    return torch.as_tensor(x), torch.as_tensor(lens), torch.as_tensor(lab)


@pytest.mark.parametrize("dec_model,enc_model,nc,embed,hln", [("lstm", "lstm", 0, "add", True),
                                                              ("layer_norm", "layer_norm", 0, "add", True),
                                                              ("hyper", "lstm", 3, "add", True),
                                                              ("hyper", "lstm", 0, "add", False),
                                                              ("lstm", "lstm", 3, "concat", True)])
def test_vae_loss_and_grads(dec_model, enc_model, nc, embed, hln):
    cfg = VAEConfig(enc_rnn_size=16, dec_rnn_size=24, z_size=8, num_mixture=3, max_seq_len=20, dec_model=dec_model,
                    enc_model=enc_model, hyper_num_units=12, hyper_embedding_size=4, num_classes=nc,
                    class_embed=embed, use_input_dropout=True, use_output_dropout=True, hyper_use_layer_norm=hln)
    m = SketchVAE(cfg, seed=0)
    x, lens, lab = _vae_batch(cfg)
    out = m.loss(x, lens, lab if nc else None, kl_weight=0.3, train=True, seed=2)
    assert set(out) == {"cost", "r_cost", "kl_cost", "shape_cost", "pen_cost"}
    assert abs(float(out["cost"]) - float(out["r_cost"] + 0.3 * out["kl_cost"])) < 1e-5
    assert float(out["kl_cost"]) >= cfg.kl_tolerance - 1e-7
    assert abs(float(out["r_cost"]) - float(out["shape_cost"] + out["pen_cost"])) < 1e-5
    out["cost"].backward()
    for n, p in m.named_parameters():
        assert p.grad is not None and torch.isfinite(p.grad).all(), n


def test_vae_kl_floor_blocks_gradient():
    cfg = VAEConfig(enc_rnn_size=16, dec_rnn_size=16, z_size=4, num_mixture=2, max_seq_len=16, kl_tolerance=100.0)
    m = SketchVAE(cfg, seed=0)
    x, lens, lab = _vae_batch(cfg)
    out = m.loss(x, lens, None, kl_weight=1.0, train=False, eps=torch.zeros(4, 4))
    assert float(out["kl_cost"]) == 100.0
    out["kl_cost"].backward() if out["kl_cost"].requires_grad else None
    assert all(p.grad is None or float(p.grad.abs().sum()) == 0 for p in m.encoder.parameters())


@pytest.mark.parametrize("dec_model", ["lstm", "layer_norm", "hyper"])
def test_vae_initial_state_layout(dec_model):
    cfg = VAEConfig(enc_rnn_size=8, dec_rnn_size=10, z_size=4, num_mixture=2, dec_model=dec_model,
                    hyper_num_units=6, hyper_embedding_size=3)
    m = SketchVAE(cfg, seed=0)
    z = torch.randn(3, 4)
    st = m.initial_state(z, 3, "cpu")
    full = torch.tanh(z @ m.init_w + m.init_b)
    if dec_model == "lstm":        # [c, h]
        assert torch.equal(st[1], full[:, :10]) and torch.equal(st[0], full[:, 10:])
    elif dec_model == "layer_norm":  # [h, c]
        assert torch.equal(st[0], full[:, :10]) and torch.equal(st[1], full[:, 10:])
    else:                           # [h, hh, c, hc]
        assert torch.equal(st[0], full[:, :10]) and torch.equal(st[1], full[:, 16:26])
        assert torch.equal(st[2], full[:, 10:16]) and torch.equal(st[3], full[:, 26:])


def test_vae_decode_step_matches_sequence():
    cfg = VAEConfig(enc_rnn_size=8, dec_rnn_size=16, z_size=4, num_mixture=2, dec_model="hyper",
                    hyper_num_units=8, hyper_embedding_size=4)
    m = SketchVAE(cfg, seed=0).eval()
    z = torch.randn(2, 4)
    x = torch.randn(5, 2, 5)
    st = m.initial_state(z, 2, "cpu")
    with torch.no_grad():
        out, _ = m.decode(x, z, st, train=False, seed=0)
        zs = m.head(out).view(5, 2, -1)
        s = st
        for t in range(5):
            zh, s = m.decode_step(x[t], z, s)
            assert torch.allclose(zh, zs[t], atol=1e-5)


def test_unconditional_vae_has_no_encoder_cost():
    cfg = VAEConfig(conditional=False, dec_rnn_size=16, num_mixture=2, max_seq_len=16)
    m = SketchVAE(cfg, seed=0)
    x, lens, _ = _vae_batch(cfg)
    out = m.loss(x, lens, None, train=True)
    assert float(out["kl_cost"]) == 0.0
    out["cost"].backward()


def test_ops_backend_switch():
    ops.set_backend("torch")
    assert ops.get_backend() == "torch"
    ops.set_backend("auto")
    with pytest.raises(ValueError):
        ops.set_backend("cuda")
    assert not ops.use_hip(torch.zeros(1))
