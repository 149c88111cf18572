#!/usr/bin/env python3
"""BASELINE config 5 gate: fp8 gate GEMMs on CDNA4's block-scaled fp8 MFMA
(csrc/skinny_gemm.hip, v_mfma_scale_f32_16x16x128_f8f6f4) for the dec=2048
HyperLSTM.

1. trains vae_large (bf16, synthetic stroke-5, random init) for --steps
   steps so the recurrence carries trained structure (not the random-init
   state, where NLL barely depends on the GEMM precision);
2. evaluates the held-out recon NLL of that model with the decoder's GEMM
   operands in bf16 and in fp8 (the inference path: e4m3 weights with
   per-column scales, e4m3 activations x64);
3. times the hipGraph-captured temperature-sampled decode (GraphDecoder) at
   --batch rows in bf16 and fp8.

Prints one JSON line (profiles/r4/fp8_gate.json).
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
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--decode-steps", type=int, default=250)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from sketch_rnn_amd import ops
    from sketch_rnn_amd.config import PRESETS
    from sketch_rnn_amd.data.dataset import StrokeDataset
    from sketch_rnn_amd.data.synthetic import synthetic_corpus
    from sketch_rnn_amd.ops import gemm
    from sketch_rnn_amd.sample.sampler import GraphDecoder
    from sketch_rnn_amd.train.trainer import VAETrainer

    ops.set_backend("hip")
    cfg = PRESETS["vae_large"].replace(save_every=0)
    strokes, labels = synthetic_corpus(3000, seed=1234, max_len=cfg.max_seq_len)
    n_test = 300
    train = StrokeDataset(strokes[n_test:], cfg.batch_size, cfg.max_seq_len, random_scale_factor=cfg.random_scale_factor,
                          augment_stroke_prob=cfg.augment_stroke_prob, labels=labels[n_test:], seed=7)
    scale = train.normalize()
    test = StrokeDataset(strokes[:n_test], cfg.batch_size, cfg.max_seq_len, labels=labels[:n_test], seed=8)
    test.normalize(scale)
    tr = VAETrainer(cfg, train, None, test, device="cuda", save_dir="/tmp/skr_fp8_gate", log=lambda s: None,
                    compute_dtype="bf16")
    t0 = time.time()
    tr.train(num_steps=a.steps, log_every=100)
    torch.cuda.synchronize()
    train_s = time.time() - t0
    res = {"train_steps": a.steps, "train_s": round(train_s, 1)}
    for dt in ("bf16", "fp8"):
        ops.set_compute_dtype(dt)
        gemm.invalidate_derived()
        ev = tr.evaluate(test)
        res["test_recon_nll_" + dt] = round(ev["r_cost"], 5)
    res["nll_gap_rel"] = round((res["test_recon_nll_fp8"] - res["test_recon_nll_bf16"]) /
                               abs(res["test_recon_nll_bf16"]), 5)
    model = tr.model.eval()
    for dt in ("bf16", "fp8"):
        ops.set_compute_dtype(dt)
        gemm.invalidate_derived()
        dec = GraphDecoder(model, a.batch, a.decode_steps, temperature=0.5)
        z = torch.randn(a.batch, cfg.z_size, device="cuda")
        dec.run(seed=1, z=z)        # capture + warm
        torch.cuda.synchronize()
        ts = []
        for r in range(a.reps):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            dec.run(seed=2 + r, z=z)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t1)
        best = min(ts)
        res["decode_ms_per_step_" + dt] = round(1e3 * best / a.decode_steps, 4)
        res["decode_strokes_per_s_" + dt] = round(a.batch * a.decode_steps / best, 1)
    res["fp8_decode_speedup"] = round(res["decode_ms_per_step_bf16"] / res["decode_ms_per_step_fp8"], 4)
    res.update({"config": "vae_large dec 2048 HyperLSTM", "batch": a.batch, "decode_steps": a.decode_steps,
                "data": "synthetic stroke-5, trained from random init"})
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
