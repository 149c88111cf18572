"""MX-fp8 kernels (csrc/mx8_gemm.hip) against PyTorch: the quantizers
against a PyTorch transcription (torch's OCP float8_e4m3fn rounding), byte
for byte; the block-scaled GEMM against the fp64 product of the dequantized
operands -- block magnitudes spread over many binades, so a scale applied to
the wrong lane / K-block / K-step shows up at once."""
import pytest
import torch

from sketch_rnn_amd.ops import mx8
from sketch_rnn_amd.utils import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _spread(R, K, g):
    """Random values with per-(row, 32-block) magnitudes 2^-8 .. 2^8."""
    x = torch.randn(R, K, device=DEV, generator=g)
    e = torch.randint(-8, 9, (R, K // 32, 1), device=DEV, generator=g).float()
    return (x.view(R, K // 32, 32) * torch.exp2(e)).view(R, K)


@pytest.mark.parametrize("K,N", [(256, 128), (2048, 8192)])
def test_quant_t_matches_torch(K, N):
    native.require_hip()
    g = torch.Generator(device=DEV).manual_seed(1)
    W = _spread(N, K, g).t().contiguous()          # [K, N]: blocks along K of each column
    Q, S = mx8.quant_t(W)
    qr, sr = mx8.quant_ref(W.t().contiguous())
    torch.cuda.synchronize()
    assert torch.equal(S, sr)
    assert torch.equal(Q, qr)
    # e4m3 (3 mantissa bits): error <= 1/16 of the value, or of the block's
    # subnormal step for values far below its maximum -- bounded by 1/16 of the block amax
    d = mx8.dequant(Q, S).view(N, K // 32, 32)
    wt = W.t().contiguous().view(N, K // 32, 32)
    amax = wt.abs().amax(-1, keepdim=True)
    assert float(((d - wt).abs() / amax.clamp_min(1e-30)).max()) <= 2.0 ** -4


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_quant_rows_matches_torch(dt):
    native.require_hip()
    g = torch.Generator(device=DEV).manual_seed(2)
    A = _spread(37, 512, g).to(dt)
    Q, S = mx8.quant_rows(A)
    qr, sr = mx8.quant_ref(A.float())
    torch.cuda.synchronize()
    assert torch.equal(S, sr) and torch.equal(Q, qr)


@pytest.mark.parametrize("M,N,K", [(100, 256, 512), (128, 128, 2048), (1024, 8192, 2048), (37, 384, 1024)])
def test_mx8_gemm_vs_fp64(M, N, K):
    native.require_hip()
    g = torch.Generator(device=DEV).manual_seed(3)
    A8, SA = mx8.quant_rows(_spread(M, K, g))
    W8, SW = mx8.quant_t(_spread(N, K, g).t().contiguous())
    C = mx8.gemm(A8, SA, W8, SW)
    ref = mx8.dequant(A8, SA).double() @ mx8.dequant(W8, SW).double().t()
    torch.cuda.synchronize()
    # exact products, accumulated in the MFMA's adder (measured ~4e-5 of the
    # row-column magnitude with block magnitudes 2^-8 .. 2^8): relative to
    # sum |a| |w| -- a scale applied to the wrong block / lane / K-step is O(0.1 .. 1)
    mag = mx8.dequant(A8, SA).double().abs() @ mx8.dequant(W8, SW).double().abs().t()
    err = ((C.double() - ref).abs() / mag.clamp_min(1e-300)).max().item()
    assert err < 2e-4, err


def _teacher_forced_heads(m, fp8, B, T, g):
    """Head outputs of the fused HyperLSTM step decoder fed ground-truth-like
    strokes (teacher forcing through step_fused with smp=None)."""
    from sketch_rnn_amd.sample.hyper_step import HyperStepDecoder
    cfg = m.cfg
    st = HyperStepDecoder(m, B, torch.device(DEV), fp8=fp8)
    assert st.fused and st.fp8 == fp8
    z = torch.randn(B, cfg.z_size, device=DEV, generator=g)
    zc = m.condition(z, None, B, DEV)
    st.begin(zc, m.initial_state(zc, B, DEV))
    xs = torch.zeros(T, B, 5, device=DEV)
    xs[:, :, :2] = torch.randn(T, B, 2, device=DEV, generator=g) * 0.3
    xs[:, :, 2] = 1.0
    outs = []
    for t in range(T):
        st.X.copy_(xs[t])
        st.step_fused(t, None)
        st.head()
        outs.append(st.ZS.sum(0)[:, :cfg.n_out].clone() + st._w["bo"][:cfg.n_out])
    torch.cuda.synchronize()
    return torch.stack(outs)


@pytest.mark.parametrize("B", [64, 256])
def test_fp8_decode_step(B):
    """The fp8 stroke (BASELINE config 5): (1) the main cell's fp8 copy of h
    (FwdArgs::h_q8) is byte-identical to the PyTorch quantizer applied to the
    fp32 h it produced; (2) the next stroke's h W_h slab equals the fp64
    product of the dequantized operands; (3) teacher-forced head outputs stay
    near the bf16 stroke's over 12 strokes (fp8 rounding compounds through the
    recurrence: loose bound, the quality gate is scripts/fp8_decode_eval.py);
    (4) the graph decoder samples complete sketches on it."""
    from sketch_rnn_amd import ops
    from sketch_rnn_amd.config import VAEConfig
    from sketch_rnn_amd.models.vae import SketchVAE
    from sketch_rnn_amd.sample import sampler as SM
    from sketch_rnn_amd.sample.hyper_step import HyperStepDecoder
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    try:
        cfg = VAEConfig(enc_rnn_size=64, dec_rnn_size=512, z_size=32, dec_model="hyper", hyper_num_units=256,
                        hyper_embedding_size=32, num_classes=0, max_seq_len=24)
        m = SketchVAE(cfg, seed=2).to(DEV).eval()
        with torch.no_grad():   # off the degenerate init: carry signal through W_h
            m.dec.W_h.add_(torch.randn_like(m.dec.W_h) * 0.02)
        H = cfg.dec_rnn_size
        g = torch.Generator(device=DEV).manual_seed(4)
        st = HyperStepDecoder(m, B, torch.device(DEV), fp8=True)
        assert st.fp8 and st.S_m == 1
        zc = m.condition(torch.randn(B, cfg.z_size, device=DEV, generator=g), None, B, DEV)
        st.begin(zc, m.initial_state(zc, B, DEV))
        st.X.copy_(torch.tensor([0.1, -0.2, 1.0, 0.0, 0.0], device=DEV).expand(B, 5))
        st.step_fused(0, None)
        torch.cuda.synchronize()
        q, sc = mx8.quant_ref(st.Hout)
        assert torch.equal(st.A8, q) and torch.equal(st.SA, sc)
        A8, SA = st.A8.clone(), st.SA.clone()
        st.step_fused(1, None)
        torch.cuda.synchronize()
        W8, SW = st._w["Wh8"]
        ref = mx8.dequant(A8, SA).double() @ mx8.dequant(W8, SW).double().t()
        mag = mx8.dequant(A8, SA).double().abs() @ mx8.dequant(W8, SW).double().abs().t()
        assert float(((st.RM[0].double() - ref).abs() / mag.clamp_min(1e-30)).max()) < 2e-4
        zb = _teacher_forced_heads(m, False, B, 12, torch.Generator(device=DEV).manual_seed(5))
        zf = _teacher_forced_heads(m, True, B, 12, torch.Generator(device=DEV).manual_seed(5))
        rel = float((zf - zb).norm() / zb.norm())
        assert 0 < rel < 0.15, rel
        dec = SM.GraphDecoder(m, batch=B, steps=24, temperature=0.5, fp8=True)
        s, lens = dec.run(seed=1)
        torch.cuda.synchronize()
        assert dec._steppers()[0][2].fp8
        assert torch.isfinite(s).all() and bool((lens >= 1).all())
    finally:
        ops.set_backend("auto")
        ops.set_compute_dtype("fp32")
