"""The fused VAE latent node (ops/latent.py, csrc/latent.hip) against the
same model with the latent layer as separate torch ops (SKR_LATENT_FUSED=0
path): loss terms and every parameter gradient, with hashed noise and with
explicit eps, KL above and below its tolerance (the clamp's gradient)."""
import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.models import vae as V

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _restore():
    yield
    V.LATENT_FUSED = True
    ops.set_backend("auto")
    ops.set_compute_dtype("fp32")


def _batch(B, T, seed):
    from sketch_rnn_amd.data.synthetic import synthetic_corpus
    from sketch_rnn_amd.data.dataset import StrokeDataset
    strokes, labels = synthetic_corpus(4 * B, seed=seed, max_len=T)
    ds = StrokeDataset(strokes, B, T, seed=1)
    ds.normalize()
    s, l, _ = ds.get_batch(0)
    return torch.as_tensor(s).float().to(DEV), torch.as_tensor(l).long().to(DEV)


@pytest.mark.parametrize("dec_model,kl_tol,given_eps", [("hyper", 0.2, False), ("lstm", 1e-6, True),
                                                        ("layer_norm", 1e-6, False)])
def test_fused_latent_matches_torch_ops(dec_model, kl_tol, given_eps):
    from sketch_rnn_amd.config import VAEConfig
    cfg = VAEConfig(enc_rnn_size=256, dec_rnn_size=512, dec_model=dec_model, z_size=64, max_seq_len=40,
                    batch_size=32, kl_tolerance=kl_tol, hyper_num_units=256 if dec_model == "hyper" else 256)
    m = V.SketchVAE(cfg, seed=3).to(DEV)
    with torch.no_grad():   # make the latent path carry signal at init
        m.encoder.mu_w.mul_(300.0)
        m.encoder.sig_w.mul_(300.0)
        m.init_w.mul_(300.0)
    strokes, lengths = _batch(cfg.batch_size, cfg.max_seq_len, 5)
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    eps = torch.randn(cfg.batch_size, cfg.z_size, device=DEV) if given_eps else None
    seed = torch.tensor([9], device=DEV)
    res = {}
    for fused in (True, False):
        V.LATENT_FUSED = fused
        m.zero_grad(set_to_none=True)
        out = m.loss(strokes, lengths, kl_weight=0.7, train=True, seed=seed, eps=eps)
        out["cost"].backward()
        res[fused] = ({k: float(v) for k, v in out.items()},
                      {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None})
    (of, gf), (ou, gu) = res[True], res[False]
    for k in ("cost", "r_cost", "kl_cost"):
        assert abs(of[k] - ou[k]) <= 1e-4 * max(1.0, abs(ou[k])), (k, of[k], ou[k])
    assert set(gf) == set(gu)
    for n in gu:
        d = float((gf[n] - gu[n]).norm() / gu[n].norm().clamp_min(1e-12))
        assert d < 1e-2, (n, d)
