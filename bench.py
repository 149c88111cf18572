#!/usr/bin/env python3
"""Headline benchmark: seq2seq-VAE training throughput (strokes/s, whole job).

Config (BASELINE.json "large"): bidirectional-LSTM encoder 512, HyperLSTM
decoder 2048 (hyper 256 / embed 32, LayerNorm), z = 128, M = 20 mixtures,
batch 100 per GPU, Nmax = 250, KL annealing, recurrent dropout 0.9,
per-element gradient clip 1.0, Adam. Synthetic stroke-3 sketches (no network
in this environment) and random-init weights. Every step is a full training
step (encoder + decoder forward, backward, all-reduce, clip + Adam) over all
250 decoder positions (the pen-state loss covers every position in training
mode, so all B*Nmax positions are training targets).

Usage: ``python bench.py --gpus N --steps K --warmup W``. For N > 1 the job
runs one rank per GPU over RCCL: either the caller launches it under
``torch.distributed.run`` (WORLD_SIZE set), or this script starts that
launcher itself as a child process before anything touches the GPU and exits
with its code. Rank 0 prints one JSON line:

* ``value`` -- valid (non-padding) stroke points processed per second by the
  whole job: sum of the sketch lengths of the K timed global batches divided
  by the max-over-ranks wall time (strokes/s = sum of valid
  steps / wall time);
* ``positions_per_s`` -- all ``global_batch * Nmax`` decoder positions per
  second (the Magenta recipe trains the pen-state loss on every padded
  position too, so these are loss targets; round 1 reported this number as
  ``value``).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch_ranks(n: int) -> int:
    """Start ``n`` ranks (one per GPU) under torch.distributed.run as a child
    process and return its exit code. Runs before this process touches the
    GPU (device_count() does not initialise it on this image)."""
    import subprocess
    import torch
    ndev = torch.cuda.device_count()
    if ndev < n:
        print("bench.py: --gpus %d requested but only %d device(s) visible" % (n, ndev), file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="vae_large")
    ap.add_argument("--batch", type=int, default=100, help="per-GPU batch")
    ap.add_argument("--seq-len", type=int, default=250)
    ap.add_argument("--dtype", default="bf16", choices=["fp32", "bf16"])
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-eval", action="store_true")
    ap.add_argument("--trace", action="store_true", help="print every step's cost to stderr (syncs each step)")
    ap.add_argument("--sketches", type=int, default=2000)
    ap.add_argument("--dist-backend", default=None, help="override (default: nccl = RCCL on GPUs); "
                    "'gloo' rehearses the multi-rank path with several ranks on one GPU")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _launch_ranks(args.gpus)

    import torch
    from sketch_rnn_amd import ops
    from sketch_rnn_amd.config import PRESETS
    from sketch_rnn_amd.utils.provenance import tree_identity
    from sketch_rnn_amd.data.dataset import StrokeDataset
    from sketch_rnn_amd.data.synthetic import synthetic_corpus
    from sketch_rnn_amd.parallel import dp
    from sketch_rnn_amd.train.trainer import VAETrainer

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    device = "cuda:%d" % (local_rank % max(ndev, 1)) if torch.cuda.is_available() else "cpu"
    if device.startswith("cuda"):
        torch.cuda.set_device(torch.device(device))
    if world_env > 1:
        dp.init_from_env(backend=args.dist_backend, device=device)
    world, rank = dp.world_size(), dp.rank()
    if world != args.gpus and rank == 0:
        print("bench.py: --gpus %d but WORLD_SIZE=%d; reporting the real rank count" % (args.gpus, world),
              file=sys.stderr)
    ops.set_backend(args.backend)

    cfg = PRESETS[args.config].replace(batch_size=args.batch, max_seq_len=args.seq_len, save_every=0)
    strokes, labels = synthetic_corpus(args.sketches, seed=1234, max_len=args.seq_len,
                                       n_classes=max(cfg.num_classes, 1))
    n_test = max(args.batch, len(strokes) // 10)
    train = StrokeDataset(strokes[n_test:], args.batch, args.seq_len, random_scale_factor=cfg.random_scale_factor,
                          augment_stroke_prob=cfg.augment_stroke_prob, labels=labels[n_test:], seed=7, rank=rank)
    scale = train.normalize()
    test = StrokeDataset(strokes[:n_test], args.batch, args.seq_len, labels=labels[:n_test], seed=8)
    test.normalize(scale)

    trainer = VAETrainer(cfg, train, None, test, device=device, save_dir="/tmp/skr_bench",
                         use_graph=(not args.no_graph) and device.startswith("cuda"),
                         log=lambda s: None, compute_dtype=args.dtype)
    nparam = sum(p.numel() for p in trainer.model.parameters())

    def batch():
        return trainer.batch_to_device(train.random_batch(rank, world))

    batches = [batch() for _ in range(4)]
    # valid stroke points per global batch (every rank draws the same count of rows)
    valid = [float(dp.sum_scalar(float(b[1].sum()))) for b in batches]
    sync = torch.cuda.synchronize if device.startswith("cuda") else (lambda: None)
    for i in range(args.warmup):
        out = trainer.train_step(*batches[i % len(batches)])
        if args.trace:
            print("warmup %d cost %.6f" % (i, float(out["cost"])), file=sys.stderr)
    sync()
    dp.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        out = trainer.train_step(*batches[i % len(batches)])
        if args.trace:
            print("step %d cost %.6f" % (i, float(out["cost"])), file=sys.stderr)
    sync()
    dp.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    elapsed = dp.max_scalar(elapsed)
    if device.startswith("cuda"):
        from sketch_rnn_amd.train.trainer import check_device_faults
        check_device_faults()   # a timed-out in-launch exchange invalidates the run: fail loudly
    # global mean over ranks (reduced with the last gradient bucket) under DP
    cost = trainer.reduced_scalars()["cost"] if trainer.reducer is not None else float(out["cost"])
    recon = None
    if not args.no_eval:
        ev = trainer.evaluate(test)      # the whole held-out split (test.num_batches batches)
        recon = ev["r_cost"]
    probe = next(trainer.model.parameters())
    backend_resolved = "hip" if ops.use_hip(probe) else "torch"
    hip_lib = None
    if backend_resolved == "hip":
        from sketch_rnn_amd.utils import native
        hip_lib = native.hip_lib_stamp()
    global_batch = args.batch * world
    positions_per_s = global_batch * args.seq_len * args.steps / elapsed
    value = sum(valid[i % len(valid)] for i in range(args.steps)) / elapsed
    if rank == 0:
        # the headline metric string names the BASELINE.json config; other
        # presets say which model they measured
        metric = "train strokes/sec (whole node) + test recon NLL, enc512/dec2048 QuickDraw" \
            if args.config == "vae_large" else "train strokes/sec (whole node) + test recon NLL, %s (enc%d/dec%d %s)" % (
                args.config, cfg.enc_rnn_size, cfg.dec_rnn_size, cfg.dec_model)
        rec = {
            "metric": metric,
            "value": round(value, 1),
            "unit": "strokes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic stroke-3 sketches (QuickDraw-like lengths, Nmax=%d), random-init weights" % args.seq_len,
            "config": {
                "model": "seq2seq-VAE %s: enc %d biLSTM / dec %d %s (hyper %d, emb %d), z %d, M=%d, %d params" % (
                    args.config, cfg.enc_rnn_size, cfg.dec_rnn_size, cfg.dec_model, cfg.hyper_num_units,
                    cfg.hyper_embedding_size, cfg.z_size, cfg.num_mixture, nparam),
                "global_batch": global_batch,
                "seq_len": args.seq_len,
                "parallelism": "dp%d" % world,
                "dist_backend": dp.backend() or "none",
                "world_size_observed": world,
                "backend": ops.get_backend(),
                # what "auto" resolved to on this device, and which kernel build ran
                "backend_resolved": backend_resolved,
                "hip_lib": hip_lib,
                "tree": tree_identity(),
                "hip_graph": bool(trainer.use_graph),
            },
            "positions_per_s": round(positions_per_s, 1),
            "valid_fraction": round(value / positions_per_s, 4),
            "train_cost": round(cost, 4),
            "test_recon_nll": None if recon is None else round(recon, 4),
            "test_recon_nll_note": "mean over the full synthetic test split (%d sketches) after %d random-init "
                                   "training steps: a smoke value, not a quality result (see profiles/ for "
                                   "the convergence runs)" % (test.num_batches * args.batch, args.warmup + args.steps),
        }
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    sys.exit(main())
