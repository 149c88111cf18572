"""Row-per-workgroup LayerNorm cells (csrc/row_cell.hip) vs the clustered
cells (csrc/lstm_cell.hip) and the fp32 PyTorch oracle.

The row kernels change the reduction order of the LayerNorm statistics (one
workgroup reduction instead of per-workgroup partials + an in-launch
exchange), so they are not bitwise equal to the clustered kernels. Checked:
every output and gradient is as close to the fp32 oracle as the clustered
path's (error(row) <= 1.5 error(cluster) + 1e-3 of the largest element),
and the hot shapes really launch the row kernels.
"""
import math

import pytest
import torch

from sketch_rnn_amd import ops
from sketch_rnn_amd.ops import recurrent

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _restore():
    yield
    recurrent.ROW_CELLS = "main"
    ops.set_backend("auto")
    ops.set_compute_dtype("fp32")
    torch.cuda.synchronize()
    recurrent.check_cluster_errors(DEV)


def _compare(runs, names):
    for i, n in enumerate(names):
        ref = runs["ref"][i].float()
        scale = max(ref.abs().max().item(), 1e-3)
        e_r = (runs["row"][i].float() - ref).abs().max().item()
        e_c = (runs["cluster"][i].float() - ref).abs().max().item()
        assert e_r <= 1.5 * e_c + 1e-3 * scale, (n, e_r, e_c, scale)


def _arms(run):
    runs = {}
    for name, backend, dt, row in (("ref", "torch", "fp32", "all"), ("row", "hip", "bf16", "all"),
                                   ("cluster", "hip", "bf16", "0")):
        recurrent.ROW_CELLS = row
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        before = dict(recurrent.ROW_STATS)
        runs[name] = run()
        runs[name + "_launches"] = {k: recurrent.ROW_STATS[k] - before[k] for k in before}
    return runs


@pytest.mark.parametrize("B,keep,hkeep", [(100, 0.9, 0.9), (37, 1.0, 1.0)])
def test_row_cells_hyper_vae_large_shapes(B, keep, hkeep, monkeypatch):
    """HyperLSTM at the vae_large widths (main 2048, hyper 256, embedding 32):
    all four cell launches of every forward and backward step take the row
    kernels, and the result is as close to the oracle as the clustered path
    (the hyper cell's GEMM-fused backward launch, which runs the clustered
    body, off)."""
    from test_kernels_gpu import _hyper_run, _hyper_setup, _names
    from sketch_rnn_amd.ops import hyper
    monkeypatch.setattr(hyper, "HYPER_BWD_FUSE", False)
    monkeypatch.setattr(hyper, "CHAIN", False)   # (the chained main-cell launch: test_kernels_gpu.py)
    monkeypatch.setattr(hyper, "CELL_MOD", False)   # (the hyper cell inside the modulation launch: ditto)
    T = 7
    p, x, z, st, w = _hyper_setup(6, T, B, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    runs = _arms(lambda: _hyper_run(p, x, z, st, w, keep, hkeep))
    assert runs["row_launches"] == {"row": 4 * T, "cluster": 0, "chain": 0, "chain3": 0}, runs["row_launches"]
    assert runs["cluster_launches"] == {"row": 0, "cluster": 4 * T, "chain": 0, "chain3": 0}, runs["cluster_launches"]
    _compare(runs, _names(p))


@pytest.mark.parametrize("H,nd,B,keep", [(512, 1, 100, 0.9), (256, 2, 100, 1.0), (1024, 1, 24, 0.85)])
def test_row_cells_layernorm_lstm(H, nd, B, keep, monkeypatch):
    """LayerNorm-LSTM sequences (the vae_layernorm decoder, a bidirectional LN
    encoder with per-direction LayerNorm parameters) through the row kernels."""
    monkeypatch.setattr(recurrent, "LN_CHAIN", False)   # (the chained steps: test_kernels_gpu.py)
    torch.manual_seed(1)
    T = 9
    xs = [torch.randn(T, B, 4 * H, device=DEV) for _ in range(nd)]
    Ws = [torch.randn(H, 4 * H, device=DEV) / math.sqrt(H) for _ in range(nd)]
    lns = [[torch.randn(4 * H, device=DEV).mul(0.1).add(1), torch.randn(4 * H, device=DEV).mul(0.1),
            torch.randn(H, device=DEV).mul(0.1).add(1), torch.randn(H, device=DEV).mul(0.1)] for _ in range(nd)]
    h0 = torch.randn(B, H, device=DEV) * 0.3
    c0 = torch.randn(B, H, device=DEV) * 0.3
    wts = [torch.randn(T, B, H, device=DEV) for _ in range(nd)]
    seed = torch.tensor([21], device=DEV)

    def run():
        leaves = [t.clone().requires_grad_() for t in xs + Ws + [v for ln in lns for v in ln]]
        xl, Wl, ll = leaves[:nd], leaves[nd:2 * nd], leaves[2 * nd:]
        if nd == 1:
            out, (hT, cT) = ops.lstm_sequence(xl[0], Wl[0], h0, c0, drop_keep=keep, drop_seed=seed, drop_stream=3,
                                              ln=tuple(ll))
            outs = [out]
        else:
            outs = list(ops.bilstm_sequence(xl[0], xl[1], Wl[0], Wl[1], torch.zeros_like(h0), torch.zeros_like(c0),
                                            drop_keep=keep, drop_seed=seed, ln_f=tuple(ll[:4]), ln_b=tuple(ll[4:])))
        sum((o * w).sum() for o, w in zip(outs, wts)).backward()
        torch.cuda.synchronize()
        return [o.detach() for o in outs] + [t.grad for t in leaves]

    runs = _arms(run)
    assert runs["row_launches"]["row"] == 2 * T and runs["row_launches"]["cluster"] == 0, runs["row_launches"]
    _compare(runs, ["out%d" % i for i in range(nd)] + ["leaf%d" % i for i in range(6 * nd)])


def test_default_policy_row_kernels_only_in_main_backward():
    """Default SKR_ROW_CELLS=main: the HyperLSTM main-cell backward runs the
    row kernel (the first backward step as its own launch, the rest inside
    the chained dR_hyp W_y^T launch, csrc/chain_step.hip), the other three
    cell launches per step the clustered ones (the hyper cell inside the
    modulation launch, hyper.CELL_MOD, is off)."""
    from test_kernels_gpu import _hyper_run, _hyper_setup
    from sketch_rnn_amd.ops import hyper
    T = 3
    p, x, z, st, w = _hyper_setup(2, T, 100, 5, 16, 2048, 256, 32, jitter=0.02, state=0.1)
    recurrent.ROW_CELLS = "main"
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    before = dict(recurrent.ROW_STATS)
    n0 = hyper.CELL_MOD_STATS["launches"]
    _hyper_run(p, x, z, st, w)
    assert {k: recurrent.ROW_STATS[k] - before[k] for k in before} == {"row": 1, "chain": T - 1, "chain3": 0, "cluster": 3 * T}
    assert hyper.CELL_MOD_STATS["launches"] - n0 == 0
