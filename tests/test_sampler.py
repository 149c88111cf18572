"""Sampling (R14, R17, N10) on CPU: reference-sampler quirks, distribution
tests of the batched sampler math (chi-square on categorical draws, moments
of the 2-D Gaussian), and the batched decoder's CPU path."""
import math
import random

import numpy as np
import pytest
import torch

from sketch_rnn_amd.config import RefConfig, VAEConfig
from sketch_rnn_amd.models.reference import SketchRNN
from sketch_rnn_amd.models.vae import SketchVAE
from sketch_rnn_amd.sample import sampler as SM


def test_get_pi_idx_underflow_is_last():
    pdf = np.array([0.2, 0.3, 0.4])  # sums to 0.9: u > 0.9 -> -1 -> numpy "last"
    assert SM._get_pi_idx(0.1, pdf) == 0
    assert SM._get_pi_idx(0.5, pdf) == 1
    assert SM._get_pi_idx(0.95, pdf) == -1


def _ref_model(M=4, H=16):
    cfg = RefConfig(rnn_size=H, num_mixture=M, keep_prob=1.0)
    return SketchRNN(cfg, seed=0)


def test_reference_sampler_shapes_and_stop():
    m = _ref_model()
    s, params = SM.sample_reference(m, num=30, temp_mixture=0.5, temp_pen=0.5, stop_if_eoc=False,
                                    rng=np.random.RandomState(0), py_rng=random.Random(0))
    assert s.shape == (30, 5) and len(params) == 30
    assert np.all(s[:, 2:].sum(1) == 1)
    # with eoc forced as the most likely pen state, the sampler stops at the first eoc and keeps it
    with torch.no_grad():
        m.output_b[0:3] = torch.tensor([-50.0, 50.0, -50.0])
    s, _ = SM.sample_reference(m, num=30, stop_if_eoc=True, rng=np.random.RandomState(0), py_rng=random.Random(0))
    assert len(s) == 1 and s[0, 3] == 1


def test_reference_pen_temperature_bug_reproduced():
    m = _ref_model()
    kw = dict(num=12, temp_mixture=1.0, stop_if_eoc=False)
    a, pa = SM.sample_reference(m, temp_pen=0.01, rng=np.random.RandomState(3), py_rng=random.Random(3), **kw)
    b, pb = SM.sample_reference(m, temp_pen=1.0, rng=np.random.RandomState(3), py_rng=random.Random(3), **kw)
    # pen pdf identical regardless of temp_pen (model.py:230 rescales pi instead)
    for x, y in zip(pa, pb):
        np.testing.assert_allclose(x[6], y[6])
    np.testing.assert_array_equal(a[:, 2:], b[:, 2:])
    c, pc = SM.sample_reference(m, temp_pen=0.01, fix_pen_temperature=True, rng=np.random.RandomState(3),
                                py_rng=random.Random(3), **kw)
    assert any(not np.allclose(x[6], y[6]) for x, y in zip(pc[2:], pb[2:]))


def test_reference_sampler_scales_offsets():
    m = _ref_model()
    a, pa = SM.sample_reference(m, num=5, rng=np.random.RandomState(1), py_rng=random.Random(1))
    m.cfg.data_scale = 1.0
    b, _ = SM.sample_reference(m, num=5, rng=np.random.RandomState(1), py_rng=random.Random(1))
    np.testing.assert_allclose(a[:, :2], b[:, :2] * 15.0, rtol=1e-5)


def _z_rows(B, M, seed=0):
    g = torch.Generator().manual_seed(seed)
    z = torch.randn(1, 3 + 6 * M, generator=g)
    z[:, 3 + 3 * M:3 + 5 * M] = -1.0  # sigma = e^-1
    return z.repeat(B, 1)


@pytest.mark.parametrize("mode,temp", [(0, 1.0), (1, 0.5)])
def test_batched_sampler_distribution(mode, temp):
    B, M = 20000, 5
    z = _z_rows(B, M)
    out = torch.zeros(B, 5)
    nx = torch.zeros(B, 5)
    done = torch.zeros(B, dtype=torch.int32)
    params = torch.zeros(B, 4)
    step = 3
    SM.mdn_sample_torch(z, M, mode, temp, False, False, 1234, step, out, nx, done, params)
    pi = torch.softmax(z[0, 3:3 + M] / temp, -1).numpy()
    counts = np.bincount(params[:, 0].long().numpy(), minlength=M)
    chi2 = float((((counts - B * pi) ** 2) / (B * pi)).sum())
    assert chi2 < 25.0, (chi2, counts, B * pi)  # df=4, p ~ 5e-5
    k = int(np.argmax(counts))
    sel = params[:, 0].long() == k
    x = nx[sel, :2].double()
    mu = torch.tensor([z[0, 3 + M + k], z[0, 3 + 2 * M + k]]).double()
    s = math.exp(-1.0) * (temp if mode == 1 else 1.0)
    rho = math.tanh(float(z[0, 3 + 5 * M + k]))
    n = x.shape[0]
    assert torch.allclose(x.mean(0), mu, atol=5 * s / math.sqrt(n))
    cov = torch.cov(x.T)
    assert abs(float(cov[0, 0]) - s * s) < 0.08 * s * s
    assert abs(float(cov[1, 1]) - s * s) < 0.08 * s * s
    assert abs(float(cov[0, 1]) / s / s - rho) < 0.05
    pp = torch.softmax(z[0, 0:3] / (temp if mode == 1 else 1.0), -1).numpy()
    pc = np.bincount(params[:, 1].long().numpy(), minlength=3)
    assert float((((pc - B * pp) ** 2) / (B * pp)).sum()) < 20.0


def test_batched_sampler_greedy_and_done_padding():
    B, M = 6, 3
    z = _z_rows(B, M, seed=2)
    out, nx = torch.zeros(B, 5), torch.zeros(B, 5)
    done = torch.tensor([0, 1, 0, 1, 0, 0], dtype=torch.int32)
    SM.mdn_sample_torch(z, M, 1, 1.0, True, False, 0, 0, out, nx, done)
    k = int(torch.argmax(z[0, 3:3 + M]))
    assert torch.allclose(nx[:, 0], z[:, 3 + M + k]) and torch.allclose(nx[:, 1], z[:, 3 + 2 * M + k])
    np.testing.assert_array_equal(out[1].numpy(), [0, 0, 0, 0, 1])  # finished rows: end padding
    np.testing.assert_array_equal(out[0].numpy(), nx[0].numpy())


def test_graph_decoder_cpu_reference_and_vae():
    m = _ref_model()
    dec = SM.GraphDecoder(m, batch=4, steps=10, temperature=0.5)
    s, lens = dec.run(seed=3)
    s2, lens2 = dec.run(seed=3)
    assert s.shape == (4, 10, 5) and torch.equal(s, s2) and torch.equal(lens, lens2)
    assert torch.all(s[:, :, 2:].sum(-1) == 1)
    cfg = VAEConfig(enc_rnn_size=16, dec_rnn_size=32, z_size=8, num_mixture=3, max_seq_len=12, dec_model="hyper",
                    hyper_num_units=16, hyper_embedding_size=4, num_classes=3)
    vm = SketchVAE(cfg, seed=0).eval()
    dec = SM.GraphDecoder(vm, batch=3, steps=12, temperature=0.3)
    s, lens = dec.run(seed=1, labels=torch.tensor([0, 1, 2]))
    assert s.shape == (3, 12, 5) and torch.all((lens >= 1) & (lens <= 12))
    for b in range(3):
        assert torch.all(s[b, lens[b]:, 4] == 1)


def _stop_biased_vae(bias):
    cfg = VAEConfig(enc_rnn_size=16, dec_rnn_size=32, z_size=8, num_mixture=3, max_seq_len=40, dec_model="hyper",
                    hyper_num_units=16, hyper_embedding_size=4)
    vm = SketchVAE(cfg, seed=0).eval()
    ob = [p for n, p in vm.named_parameters() if n.endswith("output_b")][0]
    with torch.no_grad():
        ob[2] += bias            # the end-of-sketch pen logit (stroke-5 p3): sketches end after a few strokes
    return vm


def test_graph_decoder_early_exit_equals_full_decode():
    """Chunked decode with the all-done exit (reference model.py:254-257,
    stop_if_eoc): the emitted sketches and lengths are identical to the
    full-length decode, and the decode stops well before N once every row
    has drawn its end-of-sketch stroke."""
    vm = _stop_biased_vae(3.0)
    full = SM.GraphDecoder(vm, batch=6, steps=40, temperature=0.4, chunk=4, early_exit=False)
    early = SM.GraphDecoder(vm, batch=6, steps=40, temperature=0.4, chunk=4, early_exit=True)
    for seed in (1, 2, 3):
        sf, lf = full.run(seed=seed)
        early.out.fill_(7.0)     # stale contents from an earlier run must not survive the exit
        se, le = early.run(seed=seed)
        assert full.steps_run == 40 and early.steps_run < 40, early.steps_run
        assert early.steps_run % 4 == 0 and early.steps_run >= int(le.max())
        assert torch.equal(lf, le) and torch.equal(sf, se), seed
    # a chunk size that does not divide N
    odd = SM.GraphDecoder(vm, batch=6, steps=40, temperature=0.4, chunk=7)
    so, lo = odd.run(seed=2)
    sf, lf = full.run(seed=2)
    assert torch.equal(so, sf) and torch.equal(lo, lf)
