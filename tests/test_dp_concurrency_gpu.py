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


@pytest.mark.parametrize("hog", HOGS, ids=[h[0] for h in HOGS])
@pytest.mark.parametrize("which", ["persist_encoder", "clustered_hyper"])
def test_handoff_kernels_survive_concurrent_occupancy(which, hog):
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    run = _encoder() if which == "persist_encoder" else _hyper()
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
    print(json.dumps({"kernels": which, "hog": name, "hog_ms": us / 1e3, "solo_ms": round(solo_ms, 2),
                      "with_hog_ms": round(both_ms, 2)}))
