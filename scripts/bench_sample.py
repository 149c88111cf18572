#!/usr/bin/env python3
"""Generation throughput: temperature-sampled decode of the VAE decoder.

Compares (a) the HIP-graph batched decoder (``GraphDecoder``: decoder step
kernels + MDN head + device sampler kernel, N steps captured once and
replayed) against (b) the reference-style host loop (one sketch at a time,
one device round trip per stroke). Prints one JSON line.

usage: python scripts/bench_sample.py [--config vae_large] [--batch 256] [--steps 250]
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
    model = SketchVAE(cfg, seed=0).cuda().eval()
    dec = GraphDecoder(model, a.batch, a.steps, a.temperature)
    dec.run(seed=0)  # capture
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(a.reps):
        s, lens = dec.run(seed=r + 1)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    graph_sps = a.batch * a.steps / dt
    # host loop comparator (reference-style: one sketch, one round trip per stroke)
    t0 = time.perf_counter()
    sample_vae(model, a.host_steps, a.temperature, rng=np.random.RandomState(0))
    torch.cuda.synchronize()
    hdt = time.perf_counter() - t0
    host_sps = a.host_steps / hdt
    print(json.dumps({"metric": "sampled strokes/sec (temperature %.2f)" % a.temperature, "config": a.config,
                      "dtype": a.dtype, "batch": a.batch, "steps": a.steps,
                      "graph_decoder_strokes_per_s": round(graph_sps, 1),
                      "graph_decoder_ms_per_step": round(1000 * dt / a.steps, 4),
                      "host_loop_strokes_per_s": round(host_sps, 1),
                      "speedup": round(graph_sps / host_sps, 1),
                      "mean_len": float(lens.float().mean())}), flush=True)


if __name__ == "__main__":
    main()
