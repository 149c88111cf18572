"""Wide persistent LayerNorm-LSTM forward (csrc/lstm_wide.hip): one launch per
sequence with W_h resident in LDS over the whole chip. Checked against

* the per-step LN cell kernels (same bf16 operands): outputs, final state and
  every gradient -- the backward runs the per-step reverse kernels on the
  wide kernel's saves, so this also checks the saves;
* the fp32 PyTorch oracle (bf16 tolerances);
* itself captured in a HIP graph and replayed (bitwise) -- xfail: runs of
  the opt-in kernel differ in the last bits now and then (open ordering
  issue, csrc/lstm_wide.hip STATUS).
"""
import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.ops import recurrent

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _restore():
    yield
    ops.set_backend("auto")
    ops.set_compute_dtype("fp32")
    recurrent.WIDE_ENABLED = False
    torch.cuda.synchronize()
    recurrent.check_cluster_errors(DEV)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _inputs(T, B, H, seed=0):
    g = torch.Generator().manual_seed(seed)
    xp = (torch.randn(T, B, 4 * H, generator=g) * 0.5).to(DEV).requires_grad_()
    W = (torch.randn(H, 4 * H, generator=g) / H ** 0.5).to(DEV).requires_grad_()
    h0 = (0.3 * torch.randn(B, H, generator=g)).to(DEV).requires_grad_()
    c0 = (0.3 * torch.randn(B, H, generator=g)).to(DEV).requires_grad_()
    ln = [(1.0 + 0.1 * torch.randn(4 * H, generator=g)).to(DEV).requires_grad_(),
          (0.1 * torch.randn(4 * H, generator=g)).to(DEV).requires_grad_(),
          (1.0 + 0.1 * torch.randn(H, generator=g)).to(DEV).requires_grad_(),
          (0.1 * torch.randn(H, generator=g)).to(DEV).requires_grad_()]
    R = torch.randn(T, B, H, generator=g).to(DEV)
    return xp, W, h0, c0, ln, R


def _run(backend, dtype, wide, args):
    xp, W, h0, c0, ln, R = args
    ops.set_backend(backend)
    ops.set_compute_dtype(dtype)
    recurrent.WIDE_ENABLED = wide
    leaves = [xp, W, h0, c0] + ln
    for t in leaves:
        t.grad = None
    out, (hT, cT) = ops.lstm_sequence(xp, W, h0, c0, drop_keep=0.9, drop_seed=7, drop_stream=3, ln=tuple(ln))
    ((out * R).sum() + (hT * R[0]).sum() + (cT * R[1]).sum()).backward()
    torch.cuda.synchronize()
    return [out.detach(), hT.detach(), cT.detach()] + [t.grad.clone() for t in leaves]


NAMES = ["out", "hT", "cT", "d_xp", "d_W", "d_h0", "d_c0", "d_ln_g", "d_ln_b", "d_lnc_g", "d_lnc_b"]


@pytest.mark.parametrize("T,B,H", [(20, 100, 2048), (12, 64, 1024), (9, 37, 1024)])
def test_wide_matches_per_step_kernels(T, B, H):
    args = _inputs(T, B, H, seed=T + B)
    wide = _run("hip", "bf16", True, args)
    step = _run("hip", "bf16", False, args)
    for n, a, b in zip(NAMES, wide, step):
        assert torch.isfinite(a).all(), n
        assert _rel(a, b) < 2e-2, (n, _rel(a, b))


def test_wide_matches_oracle():
    args = _inputs(16, 100, 2048, seed=5)
    wide = _run("hip", "bf16", True, args)
    ref = _run("torch", "fp32", False, args)
    for n, a, b in zip(NAMES, wide, ref):
        assert _rel(a, b) < 5e-2, (n, _rel(a, b))


@pytest.mark.xfail(reason="open ordering issue: repeated runs differ in the last bits (lstm_wide.hip STATUS)",
                   strict=False)
def test_wide_graph_replay_matches_eager():
    from sketch_rnn_amd.train.graph import capture
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    recurrent.WIDE_ENABLED = True
    T, B, H = 24, 100, 2048
    xp, W, h0, c0, ln, _ = _inputs(T, B, H, seed=9)
    with torch.no_grad():
        def fwd():
            out, (hT, cT) = ops.lstm_sequence(xp, W, h0, c0, drop_keep=0.9, drop_seed=7, ln=tuple(ln))
            return out, cT
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fwd()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with capture(g):
            outs = fwd()
        for it in range(4):
            xp.copy_(torch.randn_like(xp) * 0.5)
            g.replay()
            got = [o.clone() for o in outs]
            ref = fwd()
            torch.cuda.synchronize()
            for a, b in zip(got, ref):
                assert torch.equal(a, b), (it, float((a - b).abs().max()))
