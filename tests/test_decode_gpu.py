"""Fused whole-sketch decoder for the reference model (csrc/decode_ref.hip,
sketch_rnn_amd/sample/fused.py):

* teacher-forced head outputs against the fp32 PyTorch step oracle
  (``SketchRNN.step`` in a loop: the reference's one-step-per-sess.run
  semantics, eoc inputs hold the fed-in state), bf16 tolerances, one and two
  layers, one row block / several / a batch split over two launches;
* sampled strokes against the PyTorch transcription of the sampler applied
  to the kernel's own head outputs, and the kernel re-run teacher-forced on
  its own samples reproduces those head outputs;
* replays are deterministic and the device seed changes the draws.
"""
import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.config import RefConfig
from sketch_rnn_amd.models.reference import SketchRNN
from sketch_rnn_amd.sample import sampler as SM
from sketch_rnn_amd.sample.fused import FusedRefDecoder, fused_decode_ok

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


def _inputs(N, B, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.zeros(N, B, 5)
    x[..., :2] = torch.randn(N, B, 2, generator=g) * 0.6
    pen = torch.multinomial(torch.tensor([0.05, 0.15, 0.8]), N * B, replacement=True, generator=g).view(N, B)
    x[..., 2:] = torch.nn.functional.one_hot(pen, 3).float()
    x[0] = 0.0
    return x


@pytest.mark.parametrize("L,B,N", [(2, 37, 30), (2, 5, 12), (1, 40, 20), (2, 230, 6)])
def test_fused_decoder_forced_matches_step_oracle(L, B, N):
    m = SketchRNN(RefConfig(rnn_size=256, num_layers=L, num_mixture=24), seed=3).to(DEV)
    assert fused_decode_ok(m)
    xs = _inputs(N, B, B * 7 + N).to(DEV)
    z = FusedRefDecoder(m, B, N).forced(xs)
    ops.set_backend("torch")
    ops.set_compute_dtype("fp32")
    st = m.zero_state(B, DEV)
    zo = []
    for t in range(N):
        zt, st = m.step(xs[t], st)
        zo.append(zt)
    zo = torch.stack(zo)
    torch.cuda.synchronize()
    err = (z - zo).abs().max().item()
    rel = ((z - zo).norm() / zo.norm()).item()
    assert rel < 1e-2 and err < 0.05 * zo.abs().max().item(), (rel, err)


def test_fused_decoder_samples_match_sampler_transcription():
    m = SketchRNN(RefConfig(rnn_size=256, num_layers=2, num_mixture=24), seed=4).to(DEV)
    B, N, temp = 48, 40, 0.5
    dec = FusedRefDecoder(m, B, N, temperature=temp)
    strokes, lengths, z = dec.run(seed=9, return_z=True)
    seed = torch.tensor([9], dtype=torch.int64, device=DEV)
    done = torch.zeros(B, dtype=torch.int32, device=DEV)
    xs = torch.zeros(N, B, 5, device=DEV)
    rows = torch.zeros(N, B, 5, device=DEV)
    for t in range(N):
        out, nx = torch.zeros(B, 5, device=DEV), torch.zeros(B, 5, device=DEV)
        SM.mdn_sample_torch(z[t], 24, 0, temp, False, False, seed, t, out, nx, done)
        rows[t] = out
        if t + 1 < N:
            xs[t + 1] = nx
    ref = rows.transpose(0, 1).clone()
    ref[:, :, 0:2] *= m.cfg.data_scale
    same = (ref[:, :, 2:] == strokes[:, :, 2:]).all(-1)
    assert same.float().mean().item() > 0.998
    assert torch.allclose(strokes[same], ref[same], rtol=1e-4, atol=1e-3)
    # the kernel fed its own draws back: teacher-forcing it on them (as
    # re-drawn by the transcription: offsets equal to float rounding of
    # exp/log/cos) reproduces z
    zf = FusedRefDecoder(m, B, N, temperature=temp).forced(xs)
    ok_rows = same.all(1)
    assert ok_rows.float().mean().item() > 0.9
    assert torch.allclose(zf[:, ok_rows], z[:, ok_rows], rtol=1e-3, atol=1e-3)
    assert (lengths >= 1).all() and (lengths <= N).all()


def test_fused_decoder_deterministic_and_seeded():
    m = SketchRNN(RefConfig(rnn_size=256, num_layers=2, num_mixture=24), seed=5).to(DEV)
    dec = FusedRefDecoder(m, 64, 50, temperature=0.3)
    a, la = dec.run(seed=1)
    b, lb = dec.run(seed=1)
    c, _ = dec.run(seed=2)
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(la, lb)
    assert not torch.equal(a, c)
    for r in range(64):   # finished rows emit eoc padding
        assert torch.all(a[r, la[r]:, 3] == 1)
