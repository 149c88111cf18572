"""Fused MDN head (csrc/mdn_head.hip): projection + loss + dL/dz in one
kernel, hand-written MFMA backward (dX, dW and the bias gradient as the extra
ones-row of the weight-gradient product). Checked against the fp32 PyTorch
oracle (dropout -> x @ W + b -> models.mdn.mdn_loss_torch) for both loss
semantics, with and without the input dropout, and with arbitrary upstream
gradients on (total, shape, pen)."""
import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.ops import mdn_hip

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _restore():
    yield
    ops.set_backend("auto")
    ops.set_compute_dtype("fp32")
    mdn_hip.FUSED_HEAD = True


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _data(N, Hd, M, mode, seed):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(N, Hd, generator=g) * 0.5).to(DEV)
    W = (torch.randn(Hd, 3 + 6 * M, generator=g) / Hd ** 0.5).to(DEV)
    b = (0.1 * torch.randn(3 + 6 * M, generator=g)).to(DEV)
    t = torch.zeros(N, 5)
    t[:, :2] = torch.randn(N, 2, generator=g) * 0.7
    pen = torch.randint(0, 3, (N,), generator=g)
    t[torch.arange(N), 2 + pen] = 1.0
    return x, W, b, t.to(DEV)


def _run(fused, x, W, b, t, M, mode, keep, coef):
    ops.set_backend("hip" if fused else "torch")
    ops.set_compute_dtype("bf16" if fused else "fp32")
    mdn_hip.FUSED_HEAD = fused
    xs, Ws, bs = (v.clone().requires_grad_() for v in (x, W, b))
    tot, shape, pen = ops.mdn_head_loss(xs, Ws, bs, t, M, mode=mode, stroke_importance=200.0, drop_keep=keep,
                                        drop_seed=5, drop_stream=7)
    (coef[0] * tot + coef[1] * shape + coef[2] * pen).backward()
    torch.cuda.synchronize()
    return [tot.detach(), shape.detach(), pen.detach(), xs.grad, Ws.grad, bs.grad]


@pytest.mark.parametrize("N,Hd,M,mode,keep", [(777, 256, 20, "magenta", 1.0), (1000, 512, 24, "reference", 0.8),
                                              (300, 2048, 20, "magenta", 0.9), (64, 256, 5, "reference", 1.0)])
def test_fused_head_matches_oracle(N, Hd, M, mode, keep):
    x, W, b, t = _data(N, Hd, M, mode, N + Hd)
    coef = (1.0, 0.0, 0.0)
    fu = _run(True, x, W, b, t, M, mode, keep, coef)
    ref = _run(False, x, W, b, t, M, mode, keep, coef)
    for n, a, r in zip(["total", "shape", "pen"], fu[:3], ref[:3]):
        assert abs(float(a) - float(r)) <= 1e-2 * abs(float(r)) + 1e-3, (n, float(a), float(r))
    for n, a, r in zip(["dx", "dW", "db"], fu[3:], ref[3:]):
        assert _rel(a, r) < 3e-2, (n, _rel(a, r))


def test_fused_head_upstream_grads():
    """Arbitrary upstream gradients on (total, shape, pen) scale the pen and
    mixture column groups of dz separately."""
    x, W, b, t = _data(500, 256, 20, "magenta", 3)
    coef = (0.7, 1.3, -0.4)
    fu = _run(True, x, W, b, t, 20, "magenta", 1.0, coef)
    ref = _run(False, x, W, b, t, 20, "magenta", 1.0, coef)
    for n, a, r in zip(["dx", "dW", "db"], fu[3:], ref[3:]):
        assert _rel(a, r) < 3e-2, (n, _rel(a, r))


def test_fused_head_is_deterministic():
    x, W, b, t = _data(2000, 512, 20, "magenta", 4)
    r1 = _run(True, x, W, b, t, 20, "magenta", 0.9, (1.0, 0.0, 0.0))
    r2 = _run(True, x, W, b, t, 20, "magenta", 0.9, (1.0, 0.0, 0.0))
    for a, c in zip(r1, r2):
        assert torch.equal(a, c)


def test_reference_model_bf16_head_grads_match_fp32():
    """The reference model's whole loss (persistent bf16 LSTM stack + fused
    head) in bf16 against the fp32 PyTorch path: output_w / output_b
    gradients within bf16 tolerances (the bf16 head path had no
    gradient check through the model)."""
    from sketch_rnn_amd.config import RefConfig
    from sketch_rnn_amd.models.reference import SketchRNN
    cfg = RefConfig(rnn_size=256, num_layers=2, num_mixture=24, keep_prob=1.0)
    m = SketchRNN(cfg, seed=2).to(DEV)
    g = torch.Generator().manual_seed(8)
    B, T = 48, 30
    x = torch.zeros(B, T, 5)
    x[..., :2] = torch.randn(B, T, 2, generator=g) * 0.5
    pen = torch.multinomial(torch.tensor([0.05, 0.1, 0.85]), B * T, replacement=True, generator=g).view(B, T)
    x[..., 2:] = torch.nn.functional.one_hot(pen, 3).float()
    y = torch.roll(x, -1, 1)
    x, y = x.to(DEV), y.to(DEV)
    grads = []
    for backend, dt in (("hip", "bf16"), ("torch", "fp32")):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        m.zero_grad(set_to_none=True)
        cost, _, _, _ = m.loss(x, y, train=False)
        cost.backward()
        torch.cuda.synchronize()
        grads.append((float(cost), m.output_w.grad.clone(), m.output_b.grad.clone()))
    (c1, w1, b1), (c2, w2, b2) = grads
    assert abs(c1 - c2) <= 1e-2 * abs(c2) + 1e-3, (c1, c2)
    assert _rel(w1, w2) < 3e-2, _rel(w1, w2)
    assert _rel(b1, b2) < 3e-2, _rel(b1, b2)
