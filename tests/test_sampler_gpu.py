"""Device sampler kernel (csrc/sampler.hip) vs its PyTorch transcription, and
the HIP-graph batched decoder (graph replay == eager decode, both through the
HIP kernels)."""
import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.config import RefConfig, VAEConfig
from sketch_rnn_amd.models.reference import SketchRNN
from sketch_rnn_amd.models.vae import SketchVAE
from sketch_rnn_amd.sample import sampler as SM
from sketch_rnn_amd.utils import native

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("mode,temp,greedy,fix_pen,step", [(0, 1.0, False, False, 0), (0, 0.4, False, True, 5),
                                                          (1, 0.5, False, False, 2), (1, 1.0, True, False, 7),
                                                          (1, 0.2, False, False, 11)])
def test_sampler_kernel_matches_torch(mode, temp, greedy, fix_pen, step):
    native.require_hip()
    B, M = 4096, 20
    g = torch.Generator(device=DEV).manual_seed(step)
    z = torch.randn(B, 3 + 6 * M, device=DEV, generator=g) * 2
    done0 = (torch.rand(B, device=DEV, generator=g) < 0.2).to(torch.int32)
    res = []
    for fn in (SM.mdn_sample_device, SM.mdn_sample_torch):
        out, nx, pr = (torch.zeros(B, 5, device=DEV), torch.zeros(B, 5, device=DEV), torch.zeros(B, 4, device=DEV))
        done = done0.clone()
        seed = torch.tensor([77], dtype=torch.int64, device=DEV)
        fn(z, M, mode, temp, greedy, fix_pen, seed, step, out, nx, done, pr)
        res.append((out, nx, done, pr))
    torch.cuda.synchronize()
    (o1, n1, d1, p1), (o2, n2, d2, p2) = res
    same = (p1[:, 0] == p2[:, 0]) & (p1[:, 1] == p2[:, 1])
    # inverse-CDF ties at float rounding may flip a handful of rows
    assert same.float().mean().item() > 0.998
    assert torch.allclose(n1[same], n2[same], rtol=1e-4, atol=1e-4)
    assert torch.allclose(o1[same], o2[same], rtol=1e-4, atol=1e-4)
    assert torch.equal(d1[same], d2[same])


def test_graph_decoder_reference_graph_equals_eager():
    native.require_hip()
    ops.set_backend("hip")
    try:
        m = SketchRNN(RefConfig(rnn_size=256, num_mixture=24), seed=0).to(DEV)
        a = SM.GraphDecoder(m, batch=64, steps=40, temperature=0.3, use_graph=True)
        b = SM.GraphDecoder(m, batch=64, steps=40, temperature=0.3, use_graph=False)
        sa, la = a.run(seed=5)
        sb, lb = b.run(seed=5)
        sa2, _ = a.run(seed=5)      # replay is deterministic
        sc, _ = a.run(seed=6)       # device seed changes the draws
        torch.cuda.synchronize()
        assert torch.equal(sa, sa2) and torch.equal(la, lb)
        assert torch.allclose(sa, sb, atol=1e-4)
        assert not torch.equal(sa, sc)
    finally:
        ops.set_backend("auto")


@pytest.mark.parametrize("dec_model", ["lstm", "layer_norm", "hyper"])
def test_graph_decoder_vae(dec_model):
    native.require_hip()
    ops.set_backend("hip")
    try:
        cfg = VAEConfig(enc_rnn_size=64, dec_rnn_size=256, z_size=32, dec_model=dec_model, hyper_num_units=64,
                        hyper_embedding_size=8, num_classes=5, max_seq_len=48)
        m = SketchVAE(cfg, seed=0).to(DEV).eval()
        lab = torch.arange(16, device=DEV) % 5
        a = SM.GraphDecoder(m, batch=16, steps=48, temperature=0.5, use_graph=True)
        b = SM.GraphDecoder(m, batch=16, steps=48, temperature=0.5, use_graph=False)
        sa, la = a.run(seed=2, labels=lab)
        sb, lb = b.run(seed=2, labels=lab)
        torch.cuda.synchronize()
        assert torch.equal(la, lb)
        assert torch.allclose(sa, sb, atol=1e-4)
        for r in range(16):
            assert torch.all(sa[r, la[r]:, 4] == 1)
    finally:
        ops.set_backend("auto")


@pytest.mark.parametrize("B", [16, 100])
def test_hyper_step_decoder_matches_decode_step(B):
    """The lean in-place HyperLSTM step (sample/hyper_step.py) against the
    generic T = 1 sequence path (SketchVAE.decode_step) on the same inputs:
    head outputs within bf16 tolerances over several strokes."""
    from sketch_rnn_amd.sample.hyper_step import HyperStepDecoder, hyper_step_ok
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    try:
        cfg = VAEConfig(enc_rnn_size=64, dec_rnn_size=512, z_size=32, dec_model="hyper", hyper_num_units=128,
                        hyper_embedding_size=16, num_classes=0, max_seq_len=16)
        m = SketchVAE(cfg, seed=1).to(DEV).eval()
        assert hyper_step_ok(m, B)
        g = torch.Generator(device=DEV).manual_seed(3)
        z = torch.randn(B, cfg.z_size, device=DEV, generator=g)
        zc = m.condition(z, None, B, DEV)
        state = m.initial_state(zc, B, DEV)
        st = HyperStepDecoder(m, B, torch.device(DEV))
        st.begin(zc, state)
        for t in range(6):
            x = torch.zeros(B, 5, device=DEV)
            x[:, :2] = torch.randn(B, 2, device=DEV, generator=g) * 0.5
            x[:, 2] = 1.0
            got = {}

            def sample(zs, ldz, nslab, slab, bias):
                got["z"] = zs[:, :, : cfg.n_out].sum(0) + bias

            st.step(x, t, sample)
            ref, state = m.decode_step(x, zc, state)
            torch.cuda.synchronize()
            rel = float((got["z"] - ref).norm() / ref.norm())
            assert rel < 2e-2, (t, rel)
    finally:
        ops.set_backend("auto")
        ops.set_compute_dtype("fp32")


def test_graph_decoder_hyper_concurrent_chunks():
    """B > 128 HyperLSTM decode: 128-row step decoders on concurrent streams
    (chunk 0 clustered LayerNorm cells, the others one workgroup per row);
    graph replay == eager, deterministic, seeded, eos padding intact."""
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    try:
        cfg = VAEConfig(enc_rnn_size=64, dec_rnn_size=512, z_size=32, dec_model="hyper", hyper_num_units=128,
                        hyper_embedding_size=16, num_classes=0, max_seq_len=32)
        m = SketchVAE(cfg, seed=4).to(DEV).eval()
        a = SM.GraphDecoder(m, batch=300, steps=32, temperature=0.5, use_graph=True)
        b = SM.GraphDecoder(m, batch=300, steps=32, temperature=0.5, use_graph=False)
        assert a._steppers() is not None and len(a._steppers()) == 3
        sa, la = a.run(seed=2)
        sa2, _ = a.run(seed=2)
        sb, lb = b.run(seed=2)
        sc, _ = a.run(seed=3)
        torch.cuda.synchronize()
        assert torch.equal(sa, sa2) and torch.equal(la, lb)
        assert torch.allclose(sa, sb, atol=1e-4)
        assert not torch.equal(sa, sc)
        for r in range(300):
            assert torch.all(sa[r, la[r]:, 4] == 1)
    finally:
        ops.set_backend("auto")
        ops.set_compute_dtype("fp32")


def _hyper256(seed=1, H=512, E=16):
    cfg = VAEConfig(enc_rnn_size=64, dec_rnn_size=H, z_size=32, dec_model="hyper", hyper_num_units=256,
                    hyper_embedding_size=E, num_classes=0, max_seq_len=32)
    return cfg, SketchVAE(cfg, seed=seed).to(DEV).eval()


@pytest.mark.parametrize("dtype,B", [("bf16", 100), ("bf16", 128), ("bf16", 96), ("bf16", 256), ("bf16", 384)])
def test_hyper_step_fused_matches_decode_step(dtype, B):
    """The four-launch stroke (decode_step.hip hyper cell + hyper_mod decode
    mode + MOD-3 main cell), teacher-forced, against the generic T = 1 path:
    head outputs within bf16 tolerances over several strokes."""
    from sketch_rnn_amd.sample.hyper_step import HyperStepDecoder
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype(dtype)
    try:
        cfg, m = _hyper256()
        g = torch.Generator(device=DEV).manual_seed(3)
        z = torch.randn(B, cfg.z_size, device=DEV, generator=g)
        zc = m.condition(z, None, B, DEV)
        state = m.initial_state(zc, B, DEV)
        st = HyperStepDecoder(m, B, torch.device(DEV))
        assert st.fused
        st.begin(zc, state)
        for t in range(6):
            x = torch.zeros(B, 5, device=DEV)
            x[:, :2] = torch.randn(B, 2, device=DEV, generator=g) * 0.5
            x[:, 2] = 1.0
            st.X.copy_(x)
            st.step_fused(t, None)
            st.head()
            got = st.ZS[:, :, : cfg.n_out].sum(0) + st._w["bo"][: cfg.n_out]
            ops.set_compute_dtype("bf16")
            ref, state = m.decode_step(x, zc, state)
            ops.set_compute_dtype(dtype)
            torch.cuda.synchronize()
            rel = float((got - ref).norm() / ref.norm())
            assert rel < 2e-2, (t, rel)
    finally:
        ops.set_backend("auto")
        ops.set_compute_dtype("fp32")


def test_hyper_step_fused_sampler_matches_slab_sampler():
    """The sampler folded into the decode hyper cell draws exactly what
    skr_mdn_sample_slabs draws from the same head slabs (stroke, next input,
    eos flags)."""
    import ctypes
    from sketch_rnn_amd.sample.hyper_step import HyperStepDecoder
    lib = native.require_hip().lib
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    try:
        cfg, m = _hyper256(seed=5)
        B, M = 100, cfg.num_mixture
        zc = m.condition(torch.randn(B, cfg.z_size, device=DEV), None, B, DEV)
        st = HyperStepDecoder(m, B, torch.device(DEV))
        x0 = torch.zeros(B, 5, device=DEV)
        x0[:, 2] = 1
        st.begin(zc, m.initial_state(zc, B, DEV), x0=x0)
        seed = torch.tensor([11], dtype=torch.int64, device=DEV)
        out = torch.zeros(B, 4, 5, device=DEV)
        done = torch.zeros(B, dtype=torch.int32, device=DEV)
        done[::7] = 1
        done_ref = done.clone()
        st.step_fused(0, None)
        st.step_fused(1, st.sample_args(0, 3, out[:, 0], done, seed, M, 1, 0.6, False, False))
        torch.cuda.synchronize()
        out_ref, nx_ref = torch.zeros(B, 5, device=DEV), torch.zeros(B, 5, device=DEV)
        rc = lib.skr_mdn_sample_slabs(st.ZS.data_ptr(), 128, st.S_o, B * 128, st._w["bo"].data_ptr(), B, M, 1, 0.6,
                                      0, 0, seed.data_ptr(), 0, 3, out_ref.data_ptr(), 5, nx_ref.data_ptr(), 5,
                                      done_ref.data_ptr(), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0
        torch.cuda.synchronize()
        assert torch.equal(out[:, 0], out_ref)
        assert torch.equal(st.X, nx_ref)
        assert torch.equal(done, done_ref)
    finally:
        ops.set_backend("auto")
        ops.set_compute_dtype("fp32")


def test_graph_decoder_hyper_fused_chunks():
    """B > 128 decode on the four-launch stroke: graph replay == eager,
    deterministic, seeded, eos padding intact."""
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    try:
        cfg, m = _hyper256(seed=4)
        a = SM.GraphDecoder(m, batch=300, steps=32, temperature=0.5, use_graph=True)
        b = SM.GraphDecoder(m, batch=300, steps=32, temperature=0.5, use_graph=False)
        stp = a._steppers()
        assert stp is not None and len(stp) == 3 and all(s[2].fused for s in stp)
        sa, la = a.run(seed=2)
        sa2, _ = a.run(seed=2)
        sb, lb = b.run(seed=2)
        sc, _ = a.run(seed=3)
        torch.cuda.synchronize()
        assert torch.equal(sa, sa2) and torch.equal(la, lb)
        assert torch.allclose(sa, sb, atol=1e-4)
        assert not torch.equal(sa, sc)
        for r in range(300):
            assert torch.all(sa[r, la[r]:, 4] == 1)
    finally:
        ops.set_backend("auto")
        ops.set_compute_dtype("fp32")


def test_graph_decoder_hyper_wide():
    """B = 256 (a multiple of 128): ONE decoder whose launches run 128-row
    blocks (grouped GEMM row blocks, hyper_mod over gridDim.z, 1024-thread
    main-cell rows) instead of concurrent 128-row chunks; graph replay ==
    eager, deterministic, eos padding intact, and the same first strokes as
    the chunked decode (identical head inputs before any split-K order
    difference can flip a draw)."""
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    try:
        cfg, m = _hyper256(seed=6)
        a = SM.GraphDecoder(m, batch=256, steps=24, temperature=0.5, use_graph=True)
        b = SM.GraphDecoder(m, batch=256, steps=24, temperature=0.5, use_graph=False)
        stp = a._steppers()
        assert stp is not None and len(stp) == 1 and stp[0][1] == 256 and stp[0][2].fused
        sa, la = a.run(seed=4)
        sa2, _ = a.run(seed=4)
        sb, lb = b.run(seed=4)
        torch.cuda.synchronize()
        assert torch.equal(sa, sa2) and torch.equal(la, lb)
        assert torch.allclose(sa, sb, atol=1e-4)
        for r in range(256):
            assert torch.all(sa[r, la[r]:, 4] == 1)
        from sketch_rnn_amd.sample import hyper_step
        hyper_step.WIDE = False
        try:
            c = SM.GraphDecoder(m, batch=256, steps=24, temperature=0.5, use_graph=False)
            assert len(c._steppers()) == 2
            sc, _ = c.run(seed=4)
        finally:
            hyper_step.WIDE = True
        torch.cuda.synchronize()
        assert torch.allclose(sa[:, 0], sc[:, 0], atol=1e-4)
    finally:
        ops.set_backend("auto")
        ops.set_compute_dtype("fp32")


@pytest.mark.parametrize("B,fused", [(128, True), (128, False), (256, True)])
def test_graph_decoder_early_exit_hyper_steppers(B, fused):
    """Chunked HIP-graph decode with the all-done exit on the in-place
    HyperLSTM step decoders (fused four-launch stroke, whose sampler draws
    stroke t inside step t + 1's launch, and the seven-launch step): the
    sketches are identical to the full-length decode of the same graphs, and
    the decode stops early once every row has ended."""
    from sketch_rnn_amd.sample import hyper_step
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    saved = hyper_step.FUSED
    try:
        hyper_step.FUSED = fused
        cfg = VAEConfig(enc_rnn_size=64, dec_rnn_size=512, z_size=32, dec_model="hyper", hyper_num_units=256,
                        hyper_embedding_size=32, num_classes=0, max_seq_len=60)
        m = SketchVAE(cfg, seed=5).to(DEV).eval()
        with torch.no_grad():
            [p for n, p in m.named_parameters() if n.endswith("output_b")][0][2] += 2.5
        full = SM.GraphDecoder(m, batch=B, steps=60, temperature=0.5, chunk=5, early_exit=False)
        early = SM.GraphDecoder(m, batch=B, steps=60, temperature=0.5, chunk=5, early_exit=True)
        assert early._steppers() is not None
        for seed in (1, 2):
            sf, lf = full.run(seed=seed)
            early.out.fill_(7.0)
            se, le = early.run(seed=seed)
            torch.cuda.synchronize()
            assert early._lag == (1 if fused else 0)
            assert early.steps_run < 60, early.steps_run
            assert torch.equal(lf, le) and torch.equal(sf, se), seed
    finally:
        hyper_step.FUSED = saved
        ops.set_backend("auto")
        ops.set_compute_dtype("fp32")


@pytest.mark.parametrize("B", [384, 1024])
def test_hyper_mod_row_block_walk_bitwise(B):
    """ops.hyper.HM_ZGRID: the wide decode's modulation launch with its row
    blocks walked by 1 or 2 workgroups per tile (P fragments loaded once)
    against one workgroup per row block: the same per-block arithmetic, so
    the head outputs of several teacher-forced strokes are bit-identical."""
    from sketch_rnn_amd.ops import hyper
    from sketch_rnn_amd.sample.hyper_step import HyperStepDecoder
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    cfg, m = _hyper256(H=2048, E=32)
    g = torch.Generator(device=DEV).manual_seed(5)
    z = torch.randn(B, cfg.z_size, device=DEV, generator=g)
    xs = []
    for t in range(4):
        x = torch.zeros(B, 5, device=DEV)
        x[:, :2] = torch.randn(B, 2, device=DEV, generator=g) * 0.5
        x[:, 2] = 1.0
        xs.append(x)
    saved = hyper.HM_ZGRID
    outs = {}
    try:
        for zg in (0, 1, 2):
            hyper.HM_ZGRID = zg
            with torch.no_grad():
                zc = m.condition(z, None, B, DEV)
                st = HyperStepDecoder(m, B, torch.device(DEV))
                assert st.fused
                st.begin(zc, m.initial_state(zc, B, DEV))
                res = []
                for t, x in enumerate(xs):
                    st.X.copy_(x)
                    st.step_fused(t, None)
                    st.head()
                    res.append(st.ZS.clone())
                torch.cuda.synchronize()
            outs[zg] = res
    finally:
        hyper.HM_ZGRID = saved
    for zg in (1, 2):
        for t in range(len(xs)):
            assert torch.equal(outs[0][t], outs[zg][t]), (zg, t)


@pytest.mark.parametrize("C", [2, 4])
def test_wide_decode_main_cell_split_rows(C):
    """sample.hyper_step.WIDE_MAIN_C: the wide decode's main cell (B = 1024
    rows) split over C workgroups per row -- more workgroups than can be
    resident at once, each row's exchange among consecutive ids -- against
    one 1024-thread workgroup per row: the same outputs up to the LayerNorm
    sums' order (1e-3 of the largest element) over several strokes, and the
    launch never raises a cluster timeout."""
    from sketch_rnn_amd.ops.recurrent import check_cluster_errors
    from sketch_rnn_amd.sample import hyper_step
    from sketch_rnn_amd.sample.hyper_step import HyperStepDecoder
    native.require_hip()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    B = 1024
    cfg, m = _hyper256(H=2048, E=32)
    g = torch.Generator(device=DEV).manual_seed(9)
    z = torch.randn(B, cfg.z_size, device=DEV, generator=g)
    xs = []
    for t in range(3):
        x = torch.zeros(B, 5, device=DEV)
        x[:, :2] = torch.randn(B, 2, device=DEV, generator=g) * 0.5
        x[:, 2] = 1.0
        xs.append(x)
    saved = hyper_step.WIDE_MAIN_C
    outs = {}
    try:
        for c in (1, C):
            hyper_step.WIDE_MAIN_C = c
            with torch.no_grad():
                zc = m.condition(z, None, B, DEV)
                st = HyperStepDecoder(m, B, torch.device(DEV))
                assert (st.clm.C == c) if c > 1 else True
                st.begin(zc, m.initial_state(zc, B, DEV))
                res = []
                for t, x in enumerate(xs):
                    st.X.copy_(x)
                    st.step_fused(t, None)
                    st.head()
                    res.append(st.ZS.sum(0).clone())
                torch.cuda.synchronize()
                check_cluster_errors(DEV)
            outs[c] = res
    finally:
        hyper_step.WIDE_MAIN_C = saved
    for t in range(len(xs)):
        a, b = outs[1][t], outs[C][t]
        assert (a - b).abs().max().item() <= 1e-3 * a.abs().max().item() + 1e-5, t

