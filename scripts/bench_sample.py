#!/usr/bin/env python3
"""Generation throughput: temperature-sampled decode of the VAE decoder.

Compares (a) the HIP-graph batched decoder (``GraphDecoder``: decoder step
kernels + MDN head + device sampler kernel, captured in chunks of steps with
an all-done exit after each chunk) against (b) the reference-style host loop
(one sketch at a time, one device round trip per stroke). Prints one JSON
line with

* ``valid_strokes_per_s`` -- sum of the sampled sketch lengths / wall time
  (the strokes a user gets; padding after a row's end-of-sketch excluded);
* ``decode_positions_per_s`` -- batch x decode steps actually run / wall time
  (row-steps the decoder computed, padding rows included);
* ``steps_run`` -- decode steps per sketch batch after the early exit.

``--train-steps N`` first trains the model N steps on synthetic sketches
(random-init models end their sketches after a handful of strokes, which
makes every throughput look like padding).

usage: python scripts/bench_sample.py [--config vae_large] [--batch 256] [--steps 250] [--train-steps 0]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="vae_large")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=250)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--temperature", type=float, default=0.5)
    ap.add_argument("--dtype", default="bf16", choices=["fp32", "bf16"])
    ap.add_argument("--host-steps", type=int, default=50, help="strokes timed for the host-loop comparator")
    ap.add_argument("--train-steps", type=int, default=0, help="train this many steps first (synthetic data)")
    ap.add_argument("--no-early-exit", action="store_true")
    ap.add_argument("--fp8", action="store_true", help="MX-fp8 h W_h in the HyperLSTM step decoder (BASELINE config 5)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from sketch_rnn_amd import ops
    from sketch_rnn_amd.config import PRESETS
    from sketch_rnn_amd.models.vae import SketchVAE
    from sketch_rnn_amd.sample.sampler import GraphDecoder, sample_vae

    ops.set_backend("hip")
    ops.set_compute_dtype(a.dtype)
    cfg = PRESETS[a.config].replace(max_seq_len=a.steps)
    train_cost = None
    if a.train_steps > 0:
        from sketch_rnn_amd.data.dataset import StrokeDataset
        from sketch_rnn_amd.data.synthetic import synthetic_corpus
        from sketch_rnn_amd.train.trainer import VAETrainer
        tcfg = cfg.replace(batch_size=100, save_every=0)
        strokes, labels = synthetic_corpus(4000, seed=1234, max_len=a.steps, n_classes=max(cfg.num_classes, 1))
        ds = StrokeDataset(strokes, tcfg.batch_size, a.steps, labels=labels, seed=7)
        ds.normalize()
        tr = VAETrainer(tcfg, ds, None, None, device="cuda", save_dir="/tmp/skr_bench_sample", log=lambda s: None,
                        compute_dtype=a.dtype)
        for _ in range(a.train_steps):
            out = tr.train_step(*tr.batch_to_device(ds.random_batch()))
        train_cost = float(out["cost"])
        model = tr.model.eval()
    else:
        model = SketchVAE(cfg, seed=0).cuda().eval()
    dec = GraphDecoder(model, a.batch, a.steps, a.temperature, early_exit=not a.no_early_exit, fp8=a.fp8)
    dec.run(seed=0)  # capture
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    total_len = total_pos = 0
    for r in range(a.reps):
        s, lens = dec.run(seed=r + 1)
        total_len += int(lens.sum())
        total_pos += a.batch * dec.steps_run
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dt = wall / a.reps
    # host loop comparator (reference-style: one sketch, one round trip per stroke)
    t0 = time.perf_counter()
    sample_vae(model, a.host_steps, a.temperature, rng=np.random.RandomState(0))
    torch.cuda.synchronize()
    hdt = time.perf_counter() - t0
    host_sps = a.host_steps / hdt
    valid_sps = total_len / wall
    print(json.dumps({"metric": "sampled valid strokes/sec (temperature %.2f)" % a.temperature, "config": a.config,
                      "dtype": a.dtype, "fp8_gemm": bool(a.fp8), "batch": a.batch, "steps": a.steps, "train_steps": a.train_steps,
                      "train_cost": train_cost, "early_exit": not a.no_early_exit,
                      "valid_strokes_per_s": round(valid_sps, 1),
                      "decode_positions_per_s": round(total_pos / wall, 1),
                      "steps_run": total_pos / a.batch / a.reps,
                      "ms_per_sketch_batch": round(1000 * dt, 3),
                      "ms_per_decode_step": round(1000 * wall / (total_pos / a.batch), 4),
                      "host_loop_strokes_per_s": round(host_sps, 1),
                      "speedup_valid_vs_host": round(valid_sps / host_sps, 1),
                      "mean_len": total_len / a.batch / a.reps}), flush=True)


if __name__ == "__main__":
    main()
