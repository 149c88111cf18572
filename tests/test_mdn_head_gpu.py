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


@pytest.mark.parametrize("N,Hd,M", [(3001, 2048, 20), (777, 512, 24)])
def test_fused_head_reads_bf16_rows(N, Hd, M):
    """With a bf16 copy of x (``x_lp``: a column slice of a wider buffer, the
    decoder's [h | hh] GEMM operand rows) the forward reads it instead of the
    fp32 x -- the same bf16 MFMA operands, so loss, dz and dX are
    bit-identical -- and [dW; db] runs on the long-K weight-gradient GEMM
    (fp32 sums in another order: close to the fp32-rows kernel and to the
    oracle)."""
    x, W, b, t = _data(N, Hd, M, "magenta", N)
    wide = torch.zeros(N, Hd + 256, device=DEV, dtype=torch.bfloat16)
    wide[:, :Hd] = x.to(torch.bfloat16)
    x_lp = wide[:, :Hd]
    res = []
    for lp in (None, x_lp):
        ops.set_backend("hip")
        ops.set_compute_dtype("bf16")
        xs, Ws, bs = (v.clone().requires_grad_() for v in (x, W, b))
        tot, shape, pen = ops.mdn_head_loss(xs, Ws, bs, t, M, mode="magenta", x_lp=lp)
        (0.7 * tot + 0.2 * shape).backward()
        torch.cuda.synchronize()
        res.append([tot.detach(), shape.detach(), pen.detach(), xs.grad, Ws.grad, bs.grad])
    for n, a, c in zip(["total", "shape", "pen", "dx"], res[0][:4], res[1][:4]):
        assert torch.equal(a, c), n
    for n, a, c in zip(["dW", "db"], res[0][4:], res[1][4:]):
        assert _rel(c, a) < 2e-3, (n, _rel(c, a))
    ref = _run(False, x, W, b, t, M, "magenta", 1.0, (0.7, 0.2, 0.0))
    for n, a, r in zip(["dW", "db"], res[1][4:], ref[4:]):
        assert _rel(a, r) < 3e-2, (n, _rel(a, r))


def test_recurrences_expose_bf16_h_rows():
    """The bf16 HyperLSTM and LSTM sequences attach their carried-h GEMM
    operand rows (``_skr_lp``) to the output: exactly the bf16 rounding of
    the returned fp32 h (what the fused head reads in its place)."""
    from sketch_rnn_amd.models import cells as C
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    torch.manual_seed(3)
    T, B, IN, H = 7, 100, 5, 512
    p = C.HyperLSTMParams(IN, H, 64, 8).to(DEV)
    x = torch.randn(T, B, IN, device=DEV)
    st = [torch.zeros(B, n, device=DEV) for n in (H, H, 64, 64)]
    out, _ = ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=4, drop_stream=9)
    assert torch.equal(out._skr_lp, out.detach().to(torch.bfloat16))
    W_h = torch.randn(H, 4 * H, device=DEV) / H ** 0.5
    xp = torch.randn(T, B, 4 * H, device=DEV)
    out2, _ = ops.lstm_sequence(xp, W_h, torch.zeros(B, H, device=DEV), torch.zeros(B, H, device=DEV),
                                drop_keep=0.9, drop_seed=4, drop_stream=9)
    lp = getattr(out2, "_skr_lp", None)   # (the persistent LSTM path keeps no such rows)
    assert lp is None or torch.equal(lp, out2.detach().to(torch.bfloat16))
