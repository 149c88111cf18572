"""Data parallelism (P1/P2) on CPU with the gloo backend, world_size 2.

* gradient averaging through the bucketed flat-arena reducer equals the
  single-process gradient of the concatenated batch;
* the VAE trainer keeps parameters bitwise identical across ranks (rank 0's
  initial weights are broadcast, every rank applies the same averaged
  update) and reports rank-averaged evaluation scalars.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from sketch_rnn_amd.parallel import dp
    assert dp.init_from_env(backend="gloo")
    return dp


def _grad_worker(rank, world, port, out_dir):
    dp = _init(rank, world, port)
    from sketch_rnn_amd.config import RefConfig
    from sketch_rnn_amd.models.reference import SketchRNN
    from sketch_rnn_amd.train.optim import FlatAdam
    torch.manual_seed(0)
    m = SketchRNN(RefConfig(rnn_size=16, num_mixture=3, keep_prob=1.0), seed=rank + 10)  # different init per rank
    opt = FlatAdam(m.parameters(), lr=0.01)
    dp.broadcast_params(opt.flat)                       # rank 0 wins
    x = torch.randn(8, 6, 5, generator=torch.Generator().manual_seed(3))
    y = torch.randn(8, 6, 5, generator=torch.Generator().manual_seed(4))
    x[..., 2:], y[..., 2:] = 0, 0
    x[..., 4], y[..., 4] = 1, 1
    sl = slice(rank * 4, rank * 4 + 4)
    opt.zero_grad()
    cost = m.loss(x[sl], y[sl], None, train=False)[0]
    cost.backward()
    red = dp.GradReducer(opt.grad, bucket_mb=0.01)      # many small buckets
    assert len(red.buckets) > 1
    red.wait(red.all_reduce(async_op=True))
    avg = dp.average_scalars({"cost": float(cost)})
    torch.save({"grad": opt.grad.clone(), "flat": opt.flat.clone(), "cost": avg["cost"]},
               os.path.join(out_dir, "r%d.pt" % rank))
    dp.barrier()
    torch.distributed.destroy_process_group()


def _vae_worker(rank, world, port, out_dir):
    dp = _init(rank, world, port)
    from sketch_rnn_amd.cli.vae_train import make_datasets
    from sketch_rnn_amd.config import VAEConfig
    from sketch_rnn_amd.train.trainer import VAETrainer
    cfg = VAEConfig(enc_rnn_size=8, dec_rnn_size=16, z_size=4, num_mixture=2, max_seq_len=24, batch_size=4,
                    save_every=0, seed=rank)  # different seeds: broadcast must still align the weights
    (tr_set, va, te), _ = make_datasets(cfg, None, 40, rank=rank)
    tr = VAETrainer(cfg, tr_set, va, te, save_dir=os.path.join(out_dir, "v"), log=lambda s: None)
    tr.train(num_steps=3, log_every=1)
    ev = tr.evaluate(te, max_batches=1)
    torch.save({"flat": tr.opt.flat.clone(), "ev": ev}, os.path.join(out_dir, "v%d.pt" % rank))
    dp.barrier()
    torch.distributed.destroy_process_group()


def _spawn(fn, tmp_path, world=2):
    port = _free_port()
    mp.start_processes(fn, args=(world, port, str(tmp_path)), nprocs=world, join=True, start_method="spawn")


def test_dp_gradient_average_equals_full_batch(tmp_path):
    _spawn(_grad_worker, tmp_path)
    r = [torch.load(tmp_path / ("r%d.pt" % k), weights_only=True) for k in range(2)]
    assert torch.equal(r[0]["flat"], r[1]["flat"]) and torch.equal(r[0]["grad"], r[1]["grad"])
    from sketch_rnn_amd.config import RefConfig
    from sketch_rnn_amd.models.reference import SketchRNN
    from sketch_rnn_amd.train.optim import FlatAdam
    m = SketchRNN(RefConfig(rnn_size=16, num_mixture=3, keep_prob=1.0), seed=10)
    opt = FlatAdam(m.parameters(), lr=0.01)
    assert torch.equal(opt.flat, r[0]["flat"])
    x = torch.randn(8, 6, 5, generator=torch.Generator().manual_seed(3))
    y = torch.randn(8, 6, 5, generator=torch.Generator().manual_seed(4))
    x[..., 2:], y[..., 2:] = 0, 0
    x[..., 4], y[..., 4] = 1, 1
    cost = m.loss(x, y, None, train=False)[0]
    cost.backward()
    assert torch.allclose(opt.grad, r[0]["grad"], atol=1e-6, rtol=1e-5)
    assert abs(float(cost) - r[0]["cost"]) < 1e-5


def test_dp_vae_trainer_ranks_stay_in_sync(tmp_path):
    _spawn(_vae_worker, tmp_path)
    v = [torch.load(tmp_path / ("v%d.pt" % k), weights_only=True) for k in range(2)]
    assert torch.equal(v[0]["flat"], v[1]["flat"])
    assert v[0]["ev"] == v[1]["ev"]


def _vae_overlap_worker(rank, world, port, out_dir):
    """Same training run with the two-phase overlapped step (decoder/head
    all-reduce in flight during the encoder backward) and with the plain
    step: the updates must agree bit for bit."""
    dp = _init(rank, world, port)
    from sketch_rnn_amd.cli.vae_train import make_datasets
    from sketch_rnn_amd.config import VAEConfig
    from sketch_rnn_amd.train.trainer import VAETrainer
    res = {}
    for mode in ("1", "0"):
        os.environ["SKR_DP_OVERLAP"] = mode
        cfg = VAEConfig(enc_rnn_size=8, dec_rnn_size=16, z_size=4, num_mixture=2, max_seq_len=24, batch_size=4,
                        save_every=0, seed=rank, num_classes=3)
        (tr_set, va, te), _ = make_datasets(cfg, None, 40, rank=rank)
        tr = VAETrainer(cfg, tr_set, va, te, save_dir=os.path.join(out_dir, "o" + mode), log=lambda s: None)
        assert tr.overlap == (mode == "1")
        if tr.overlap:
            assert len(tr.reducer.parts) == 2
        tr.train(num_steps=3, log_every=1)
        res[mode] = tr.opt.flat.clone()
    os.environ.pop("SKR_DP_OVERLAP")
    torch.save(res, os.path.join(out_dir, "o%d.pt" % rank))
    dp.barrier()
    torch.distributed.destroy_process_group()


def test_dp_overlapped_step_matches_plain_step(tmp_path):
    _spawn(_vae_overlap_worker, tmp_path)
    o = [torch.load(tmp_path / ("o%d.pt" % k), weights_only=True) for k in range(2)]
    assert torch.equal(o[0]["1"], o[0]["0"])
    assert torch.equal(o[0]["1"], o[1]["1"])
