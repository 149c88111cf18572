"""Data-parallel safety of the in-launch hand-off kernels under real
concurrency.

Under DP the trainer issues the decoder/head gradient all-reduce on RCCL's
stream while the persistent encoder backward (``lstm_persist_bwd``) runs on
the compute stream (``VAETrainer._train_step_overlap``); the clustered
LayerNorm / HyperLSTM cells run while the previous step's collectives may
still hold CUs. Those kernels need every workgroup co-resident and spin on
each other with a bounded wait, so an RCCL kernel holding CU slots could, in
principle, strand a workgroup until the wait times out.

Here an occupancy hog (``csrc/hog.hip``: RCCL-like grids, LDS footprints,
a fixed wall-time residency, always drains) is launched on a second stream
just before the kernels on the compute stream. Checked: no device fault flag,
outputs and gradients bit-identical to the solo run. The elapsed time shows
the delay: workgroups that cannot be placed wait for the hog to retire while
their placed peers spin -- far inside the spin bound even with a 200 ms hog
(an all-reduce kernel is resident for milliseconds).
"""
import ctypes
import json
import time

import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.models import cells as C
from sketch_rnn_amd.ops import recurrent
from sketch_rnn_amd.utils import native

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (name, workgroups, threads, LDS bytes per workgroup, residency us)
HOGS = [
    ("rccl_like_64x512_lds32k", 64, 512, 32 * 1024, 20000),
    ("all_cus_256x1024", 256, 1024, 0, 20000),
    ("half_chip_128x256_lds96k_200ms", 128, 256, 96 * 1024, 200000),
]


@pytest.fixture(autouse=True)
def _restore():
    yield
    ops.set_backend("auto")
    ops.set_compute_dtype("fp32")


def _hog(grid, threads, lds, us, stream):
    lib = native.require_hip()
    sink = torch.zeros(1, device=DEV)
    rc = lib.lib.skr_occupancy_hog(grid, threads, lds, us, sink.data_ptr(), stream.cuda_stream)
    assert rc == 0, rc
    return sink


def _encoder():
    """vae_large encoder shape: persistent bidirectional LSTM, H 512, B 100."""
    torch.manual_seed(3)
    T, B, H = 60, 100, 512
    xp = (torch.randn(T, 2 * B, 4 * H, device=DEV) * 0.5).requires_grad_()
    W_f = (torch.randn(H, 4 * H, device=DEV) / H ** 0.5).requires_grad_()
    W_b = (torch.randn(H, 4 * H, device=DEV) / H ** 0.5).requires_grad_()
    h0 = torch.zeros(B, H, device=DEV)
    R = [torch.randn(T, B, H, device=DEV) for _ in range(2)]

    def run():
        for t in (xp, W_f, W_b):
            t.grad = None
        of, ob = ops.bilstm_sequence_packed(xp, W_f, W_b, h0, h0, drop_keep=0.9, drop_seed=5, drop_stream=2)
        ((of * R[0]).sum() + (ob * R[1]).sum()).backward()
        return [of.detach(), ob.detach()] + [t.grad.clone() for t in (xp, W_f, W_b)]
    return run


def _hyper():
    """vae_large decoder shape: HyperLSTM H 2048 / Hh 256, B 100 (clustered LN cells)."""
    torch.manual_seed(4)
    T, B, IN, Z, H, Hh, E = 12, 100, 5, 128, 2048, 256, 32
    p = C.HyperLSTMParams(IN + Z, H, Hh, E).to(DEV)
    x = torch.randn(T, B, IN, device=DEV)
    z = torch.randn(B, Z, device=DEV, requires_grad=True)
    st = [torch.zeros(B, n, device=DEV) for n in (H, H, Hh, Hh)]
    w = torch.randn(T, B, H, device=DEV)
    params = [z] + list(p.parameters())

    def run():
        out, _ = ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=1, drop_stream=9, zc=z)
        g = torch.autograd.grad((out * w).sum(), params)
        return [out.detach()] + [t.clone() for t in g]
    return run


def _ln_lstm():
    """vae_layernorm decoder shape: LayerNorm-LSTM H 512, B 100 (chained steps
    both ways when ops.recurrent.LN_CHAIN is on)."""
    torch.manual_seed(5)
    T, B, H = 12, 100, 512
    xp = (torch.randn(T, B, 4 * H, device=DEV) * 0.5).requires_grad_()
    W = (torch.randn(H, 4 * H, device=DEV) / H ** 0.5).requires_grad_()
    h0 = torch.zeros(B, H, device=DEV)
    lnp = [torch.ones(4 * H, device=DEV).requires_grad_(), torch.zeros(4 * H, device=DEV).requires_grad_(),
           torch.ones(H, device=DEV).requires_grad_(), torch.zeros(H, device=DEV).requires_grad_()]
    seed = torch.tensor([7], device=DEV)
    w = torch.randn(T, B, H, device=DEV)
    params = [xp, W] + lnp

    def run():
        out, _ = ops.lstm_sequence(xp, W, h0, h0, drop_keep=0.9, drop_seed=seed, drop_stream=4, ln=tuple(lnp))
        g = torch.autograd.grad((out * w).sum(), params)
        return [out.detach()] + [t.clone() for t in g]
    return run


@pytest.mark.parametrize("hog", HOGS, ids=[h[0] for h in HOGS])
@pytest.mark.parametrize("which", ["persist_encoder", "clustered_hyper", "chain_bwd_main", "chain_ln"])
def test_handoff_kernels_survive_concurrent_occupancy(which, hog, monkeypatch):
    """``clustered_hyper``: the HyperLSTM with the unchained backward
    launches; ``chain_bwd_main``: the same run with the chained backward
    launch on and counted (csrc/chain_step.hip: main-cell rows spin on the
    arrival counter of producer tiles of their own launch; producers never
    wait, so a hog can only delay them) -- T - 1 = 11 chained launches per
    run; ``chain_ln``: the LayerNorm-LSTM's chained steps (skr_chain_ln_fwd /
    _bwd, the same producer-rows construction), T + T - 1 launches per run."""
    from sketch_rnn_amd.ops import hyper
    from sketch_rnn_amd.ops.recurrent import LN_CHAIN_STATS, ROW_STATS
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    monkeypatch.setattr(hyper, "CHAIN", which == "chain_bwd_main")
    monkeypatch.setattr(recurrent, "LN_CHAIN", which == "chain_ln")
    run = {"persist_encoder": _encoder, "chain_ln": _ln_lstm}.get(which, _hyper)()
    n_chain = ROW_STATS["chain"]
    n_ln = dict(LN_CHAIN_STATS)
    run()                                  # lazy setup (weight caches, occupancy queries)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ref = run()
    torch.cuda.synchronize()
    solo_ms = 1e3 * (time.perf_counter() - t0)
    recurrent.check_cluster_errors(DEV)

    name, grid, threads, lds, us = hog
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    t0 = time.perf_counter()
    with torch.cuda.stream(side):
        _hog(grid, threads, lds, us, side)
    out = run()                            # compute stream, concurrent with the hog
    torch.cuda.synchronize()
    both_ms = 1e3 * (time.perf_counter() - t0)
    recurrent.check_cluster_errors(DEV)    # raises if any in-launch wait timed out
    for a, b in zip(out, ref):
        assert torch.equal(a, b)
    if which == "chain_bwd_main":   # setup + solo + hog runs, 11 chained launches each
        assert ROW_STATS["chain"] - n_chain == 3 * 11, ROW_STATS["chain"] - n_chain
    if which == "chain_ln":         # setup + solo + hog runs, T = 12 forward and 11 backward launches each
        assert (LN_CHAIN_STATS["fwd"] - n_ln["fwd"], LN_CHAIN_STATS["bwd"] - n_ln["bwd"]) == (3 * 12, 3 * 11)
    print(json.dumps({"kernels": which, "hog": name, "hog_ms": us / 1e3, "solo_ms": round(solo_ms, 2),
                      "with_hog_ms": round(both_ms, 2)}))


def test_wait_timeout_raises_divergence_error_then_next_step_is_clean():
    """The failure path (reference divergence guard train.py:93-94):
    a persistent encoder backward whose workgroups can NOT all be resident.
    Its launch goes to a queue restricted to 16 CUs (a CU-masked stream: the
    state a co-running kernel holding the rest of the chip for longer than
    the spin bound creates; deterministic, unlike a hog on a second queue,
    whose placement against the compute queue the runtime does not promise).
    Half of the first row block is placed and waits on peers that cannot be;
    the spin bound is lowered for the test (skr_persist_set_spin_limit; the
    production bound is ~seconds). Checked: the launch drains (the timed-out
    wait poisons the launch, the rest of the grid then runs through), the
    trainer's check raises DivergenceError for that step, and after the flag
    is cleared the next step is clean and bit-identical to a normal run."""
    from sketch_rnn_amd.ops import persist
    from sketch_rnn_amd.train.trainer import DivergenceError, check_device_faults
    lib = native.require_hip().lib
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    torch.manual_seed(3)
    T, B, H = 60, 100, 512
    xp = torch.randn(T, 2 * B, 4 * H, device=DEV) * 0.5
    W = torch.randn(2, H, 4 * H, device=DEV) / H ** 0.5
    h = torch.zeros(2 * B, H, device=DEV)
    dtop = torch.randn(T, 2 * B, H, device=DEV)
    meta = (1, 2, 0.9, 2, 1.0)

    def step(stream=None):
        top, outs, s, dims = persist._fwd_launch(xp, None, None, W, None, h, h, None, None, None, 5, meta)
        if stream is not None:   # the backward launch on the restricted queue
            stream.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(stream):
                r = persist._bwd_launch(s, dims, dtop, [None, None])
            torch.cuda.current_stream().wait_stream(stream)
        else:
            r = persist._bwd_launch(s, dims, dtop, [None, None])
        torch.cuda.synchronize()
        return [top, r[0][0], r[2][0], r[5][0], r[6][0]]

    ref = step()
    check_device_faults()                  # clean before
    raw = ctypes.c_void_p()
    assert lib.skr_stream_create_cu_limited(16, ctypes.byref(raw)) == 0
    assert lib.skr_persist_set_spin_limit(1 << 12) == 0
    try:
        t0 = time.perf_counter()
        step(torch.cuda.ExternalStream(raw.value))
        ms = 1e3 * (time.perf_counter() - t0)
    finally:
        assert lib.skr_persist_set_spin_limit(0) == 0
        torch.cuda.synchronize()
        lib.skr_stream_destroy(raw.value)
    assert ms < 5000, ms                   # drained: no hang
    with pytest.raises(DivergenceError):
        check_device_faults()
    out = step()                           # the next step: flag cleared, default bound
    check_device_faults()
    for a, b in zip(out, ref):
        assert torch.equal(a, b)
    print(json.dumps({"failure_path": "persist_encoder_bwd_16cu", "step_ms": round(ms, 1)}))
