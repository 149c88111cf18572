"""Persistent LSTM sequence kernels (csrc/lstm_persist.hip) against the fp32
PyTorch oracle: forward outputs, final states and every gradient (inputs,
weights, initial state), bf16 tolerances.

* the reference decoder-only 2-layer stack (one launch for both layers, eoc
  state reset to the batch-initial state, model.py:66-95);
* the bidirectional encoder (two directions in one launch, recurrent
  dropout from the shared stateless hash).
"""
import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.ops import persist

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _restore():
    yield
    ops.set_backend("auto")
    ops.set_compute_dtype("fp32")
    persist.PERSIST_ENABLED = True
    from sketch_rnn_amd.ops.recurrent import check_cluster_errors
    torch.cuda.synchronize()
    check_cluster_errors(DEV)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


def _ref_run(m, x, state, backend, dtype):
    ops.set_backend(backend)
    ops.set_compute_dtype(dtype)
    m.zero_grad(set_to_none=True)
    st = [(h.detach().clone().requires_grad_(), c.detach().clone().requires_grad_()) for h, c in state]
    z, final = m.forward(x, st, train=False)
    g = torch.Generator(device=DEV).manual_seed(11)
    rz = torch.randn(z.shape, device=DEV, generator=g)
    rf = [torch.randn(s.shape, device=DEV, generator=g) for f in final for s in f]
    loss = (z * rz).sum() + sum((s * r).sum() for s, r in zip([s for f in final for s in f], rf))
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    for l, (h, c) in enumerate(st):
        grads["h0_%d" % l], grads["c0_%d" % l] = h.grad.clone(), c.grad.clone()
    return z.detach(), [s.detach() for f in final for s in f], grads


@pytest.mark.parametrize("B,T,with_reset", [(100, 40, True), (37, 17, False), (64, 5, True)])
def test_persistent_reference_stack_matches_oracle(B, T, with_reset):
    from sketch_rnn_amd.config import RefConfig
    from sketch_rnn_amd.models.reference import SketchRNN
    cfg = RefConfig(rnn_size=256, num_layers=2, num_mixture=4, keep_prob=1.0)
    m = SketchRNN(cfg, seed=1).to(DEV)
    g = torch.Generator().manual_seed(B + T)
    x = torch.randn(B, T, 5, generator=g) * 0.6
    pen = torch.randint(0, 3, (B, T), generator=g)
    x[..., 2:] = torch.nn.functional.one_hot(pen, 3).float()
    if not with_reset:
        x[..., 3] = 0.0
        x[..., 2] = torch.maximum(x[..., 2], 1.0 - x[..., 4])
    x = x.to(DEV)
    state = [(0.3 * torch.randn(B, 256, generator=g), 0.5 * torch.randn(B, 256, generator=g)) for _ in range(2)]
    state = [(h.to(DEV), c.to(DEV)) for h, c in state]
    z_ref, f_ref, g_ref = _ref_run(m, x, state, "torch", "fp32")
    z, f, gr = _ref_run(m, x, state, "hip", "bf16")
    assert _rel(z, z_ref) < 2e-2, _rel(z, z_ref)
    for a, b in zip(f, f_ref):
        assert _rel(a, b) < 2e-2, _rel(a, b)
    for n, ref in g_ref.items():
        assert _rel(gr[n], ref) < 4e-2, (n, _rel(gr[n], ref))


@pytest.mark.parametrize("B", [100, 192, 256])
def test_persistent_bilstm_matches_oracle(B):
    """Both encoder directions in one persistent launch vs the fp32 oracle;
    B > 128 runs 64-row blocks (2 x ceil(B / 64) x 32 workgroups <= 256 CUs)."""
    from sketch_rnn_amd.ops import persist as P
    torch.manual_seed(3)
    T, H = 30, 512
    assert P.block_rows(H, 2, 1, B) == (32 if B <= 128 else 64)
    xp = (torch.randn(T, 2 * B, 4 * H, device=DEV) * 0.5).requires_grad_()
    W_f = (torch.randn(H, 4 * H, device=DEV) / H ** 0.5).requires_grad_()
    W_b = (torch.randn(H, 4 * H, device=DEV) / H ** 0.5).requires_grad_()
    h0 = (0.2 * torch.randn(B, H, device=DEV)).requires_grad_()
    c0 = (0.2 * torch.randn(B, H, device=DEV)).requires_grad_()
    R = [torch.randn(T, B, H, device=DEV) for _ in range(2)]
    res = {}
    for backend, dt in (("torch", "fp32"), ("hip", "bf16")):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        for t in (xp, W_f, W_b, h0, c0):
            t.grad = None
        of, ob = ops.bilstm_sequence_packed(xp, W_f, W_b, h0, c0, drop_keep=0.9, drop_seed=5, drop_stream=2)
        ((of * R[0]).sum() + (ob * R[1]).sum()).backward()
        res[backend] = [of.detach(), ob.detach()] + [t.grad.clone() for t in (xp, W_f, W_b, h0, c0)]
    names = ["out_f", "out_b", "xp", "W_f", "W_b", "h0", "c0"]
    for n, a, b in zip(names, res["hip"], res["torch"]):
        assert _rel(a, b) < 4e-2, (n, _rel(a, b))


def test_persistent_bilstm_lengths_bound_each_row_block():
    """Encoder use (only h[len - 1] of each row is read): with ``lengths`` the
    persistent launch stops every 32-row block after its longest row. The
    read outputs and every gradient equal the full-length launch bit for bit
    (steps past a row's length carry zero gradient either way; the skipped
    tails are zero-filled, checked with NaN-poisoned buffers)."""
    torch.manual_seed(4)
    T, B, H = 60, 100, 512
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    g = torch.Generator().manual_seed(4)
    # row blocks with very different longest rows (17, 41, 60, 9)
    lengths = torch.cat([torch.randint(1, 18, (32,), generator=g), torch.randint(1, 42, (32,), generator=g),
                         torch.randint(1, 61, (32,), generator=g), torch.randint(1, 10, (4,), generator=g)])
    lengths[40], lengths[70], lengths[97] = 41, 60, 9
    lengths = lengths.to(DEV)
    xp = (torch.randn(T, 2 * B, 4 * H, device=DEV) * 0.5).requires_grad_()
    W_f = (torch.randn(H, 4 * H, device=DEV) / H ** 0.5).requires_grad_()
    W_b = (torch.randn(H, 4 * H, device=DEV) / H ** 0.5).requires_grad_()
    h0 = (0.2 * torch.randn(B, H, device=DEV)).requires_grad_()
    c0 = (0.2 * torch.randn(B, H, device=DEV)).requires_grad_()
    R = torch.randn(B, 2 * H, device=DEV)
    idx = (lengths - 1).clamp(min=0).view(1, B, 1).expand(1, B, H)
    res = []
    persist.POISON = True
    try:
        for lens in (None, lengths):
            for t in (xp, W_f, W_b, h0, c0):
                t.grad = None
            of, ob = ops.bilstm_sequence_packed(xp, W_f, W_b, h0, c0, drop_keep=0.9, drop_seed=5, drop_stream=2,
                                                lengths=lens)
            last = torch.cat([torch.gather(o, 0, idx).squeeze(0) for o in (of, ob)], -1)
            (last * R).sum().backward()
            torch.cuda.synchronize()
            res.append([last.detach()] + [t.grad.clone() for t in (xp, W_f, W_b, h0, c0)])
    finally:
        persist.POISON = False
    for n, a, b in zip(["last_h", "xp", "W_f", "W_b", "h0", "c0"], *res):
        assert torch.isfinite(b).all(), n
        assert torch.equal(a, b), (n, float((a - b).abs().max()))


def test_persistent_matches_per_step_kernels():
    """Same model, persistent launch vs the per-step fused kernels (both
    bf16): outputs agree to bf16 rounding of the operands."""
    from sketch_rnn_amd.config import RefConfig
    from sketch_rnn_amd.models.reference import SketchRNN
    cfg = RefConfig(rnn_size=256, num_layers=2, num_mixture=4, keep_prob=1.0)
    m = SketchRNN(cfg, seed=2).to(DEV)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(100, 60, 5, generator=g)
    x[..., 2:] = torch.nn.functional.one_hot(torch.randint(0, 3, (100, 60), generator=g), 3).float()
    x = x.to(DEV)
    state = [(torch.zeros(100, 256, device=DEV), torch.zeros(100, 256, device=DEV)) for _ in range(2)]
    z1, f1, g1 = _ref_run(m, x, state, "hip", "bf16")
    persist.PERSIST_ENABLED = False
    z2, f2, g2 = _ref_run(m, x, state, "hip", "bf16")
    assert _rel(z1, z2) < 1e-2
    for n in g1:
        assert _rel(g1[n], g2[n]) < 3e-2, (n, _rel(g1[n], g2[n]))


def test_persistent_graph_replay_matches_eager():
    """The persistent launch captured in a HIP graph and replayed with new
    inputs equals the eager launch bitwise. The hand-off buffers are filled
    with NaN before every launch (persist.POISON), so a consumer that reads a
    step before its producer published it -- e.g. because the per-launch flag
    reset was not ordered before the kernel on replay -- shows up as NaN."""
    from sketch_rnn_amd.train.graph import capture
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    persist.POISON = True
    try:
        torch.manual_seed(3)
        T, B, H = 60, 16, 256
        xp = torch.randn(T, 2 * B, 4 * H, device=DEV) * 0.5
        W_f, W_b = (torch.randn(H, 4 * H, device=DEV) / H ** 0.5 for _ in range(2))
        h0, c0 = (0.2 * torch.randn(B, H, device=DEV) for _ in range(2))

        def fwd():
            return ops.bilstm_sequence_packed(xp, W_f, W_b, h0, c0, drop_keep=0.9, drop_seed=5, drop_stream=2)

        with torch.no_grad():
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                fwd()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with capture(g):
                outs = fwd()
            for it in range(6):
                xp.copy_(torch.randn_like(xp) * 0.5)
                g.replay()
                got = [o.clone() for o in outs]
                ref = fwd()
                torch.cuda.synchronize()
                for a, b in zip(got, ref):
                    assert torch.equal(a, b), (it, float((a - b).abs().max()))
    finally:
        persist.POISON = False


@pytest.mark.parametrize("B", [100, 256])
def test_fused_encoder_last_h_matches_unfused_and_oracle(B):
    """The VAE encoder as one node (input projection + persistent biLSTM
    writing only h[len-1], ops/persist.py _PersistBiEncoder) against the
    unfused HIP path (projection, persistent biLSTM with [T, 2B, H] outputs,
    gather) -- forward bit-identical, recurrent-weight gradients bit-identical,
    projection gradients (now read from the bf16 gate gradient) close -- and
    against the fp32 torch oracle at bf16 tolerances."""
    from sketch_rnn_amd.config import VAEConfig
    from sketch_rnn_amd.models.vae import Encoder
    cfg = VAEConfig(enc_rnn_size=512, dec_rnn_size=512, z_size=64, max_seq_len=60, batch_size=B)
    gen = torch.Generator().manual_seed(2)
    enc = Encoder(cfg, gen).to(DEV)
    T = 60
    g = torch.Generator().manual_seed(3)
    x = torch.randn(T, B, 5, generator=g) * 0.5
    lengths = torch.randint(5, T + 1, (B,), generator=g)
    x, lengths = x.to(DEV), lengths.to(DEV)
    rm = torch.randn(B, cfg.z_size, device=DEV)
    rs = torch.randn(B, cfg.z_size, device=DEV)

    def run(backend, dtype, fused):
        ops.set_backend(backend)
        ops.set_compute_dtype(dtype)
        persist.BI_ENCODER = fused
        enc.zero_grad(set_to_none=True)
        mu, ps = enc(x, lengths, True, torch.tensor([7], device=DEV))
        ((mu * rm).sum() + (ps * rs).sum()).backward()
        return [mu.detach(), ps.detach()], {n: p.grad.clone() for n, p in enc.named_parameters()}

    try:
        (o_f, g_f), (o_u, g_u), (o_t, g_t) = run("hip", "bf16", True), run("hip", "bf16", False), \
            run("torch", "fp32", False)
    finally:
        persist.BI_ENCODER = True
    for a, b in zip(o_f, o_u):
        assert torch.equal(a, b)
    for n in g_f:
        if "W_h" in n or "mu_" in n or "sig_" in n:
            assert torch.equal(g_f[n], g_u[n]), n
        else:
            assert _rel(g_f[n], g_u[n]) < 1e-2, (n, _rel(g_f[n], g_u[n]))
    for a, b in zip(o_f, o_t):
        assert _rel(a, b) < 2e-2, _rel(a, b)
    for n in g_t:
        assert _rel(g_f[n], g_t[n]) < 5e-2, (n, _rel(g_f[n], g_t[n]))


@pytest.mark.parametrize("H,keep,ln", [(512, 0.9, False), (256, 1.0, False), (512, 0.9, True), (256, 1.0, True)])
def test_plain_training_layer_runs_persistent_and_matches_oracle(H, keep, ln):
    """An LSTM layer in training (the vae_small decoder: z-dependent input
    projection, initial state with a gradient) takes the persistent kernels
    (ops.lstm_sequence -> persist.lstm_stack) and matches the fp32 PyTorch
    oracle within bf16 tolerances -- outputs, dh0 / dc0, dW_h, dxp -- with the
    same hashed recurrent-dropout masks. A LayerNorm-LSTM layer (the
    vae_layernorm decoder) takes the per-step clustered cells instead and
    matches the oracle the same way, gamma / beta gradients included."""
    from sketch_rnn_amd.ops import recurrent
    B, T = 100, 48
    g = torch.Generator(device=DEV).manual_seed(H)
    xp = (torch.randn(T, B, 4 * H, device=DEV, generator=g) * 0.5)
    W = torch.randn(H, 4 * H, device=DEV, generator=g) / H ** 0.5
    h0 = torch.randn(B, H, device=DEV, generator=g) * 0.3
    c0 = torch.randn(B, H, device=DEV, generator=g) * 0.3
    w_out = torch.randn(T, B, H, device=DEV, generator=g)
    lnp = [1.0 + 0.1 * torch.randn(4 * H, device=DEV, generator=g), 0.1 * torch.randn(4 * H, device=DEV, generator=g),
           1.0 + 0.1 * torch.randn(H, device=DEV, generator=g), 0.1 * torch.randn(H, device=DEV, generator=g)]
    res = {}
    for name, backend, dt in (("ref", "torch", "fp32"), ("hip", "hip", "bf16")):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        ins = [t.detach().clone().requires_grad_() for t in [xp, W, h0, c0] + (lnp if ln else [])]
        calls = {}
        orig = persist.lstm_stack

        def spy(*a, **k):
            calls["n"] = calls.get("n", 0) + 1
            return orig(*a, **k)
        persist.lstm_stack = spy
        try:
            out, (hT, cT) = ops.lstm_sequence(ins[0], ins[1], ins[2], ins[3], drop_keep=keep, drop_seed=7,
                                              drop_stream=3, ln=tuple(ins[4:]) if ln else None)
        finally:
            persist.lstm_stack = orig
        ((out * w_out).sum() + hT.sum() + cT.sum()).backward()
        res[name] = (out.detach(), [t.grad for t in ins], calls.get("n", 0))
    assert res["hip"][2] == (0 if ln else 1), "persistent path taken: %d" % res["hip"][2]
    assert _rel(res["hip"][0], res["ref"][0]) < 2e-2
    for n, a, b in zip(("dxp", "dW_h", "dh0", "dc0", "dln_g", "dln_b", "dlnc_g", "dlnc_b"), res["hip"][1],
                       res["ref"][1]):
        assert _rel(a, b) < 4e-2, (n, _rel(a, b))
    del recurrent
