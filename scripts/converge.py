#!/usr/bin/env python3
"""Convergence-quality run: test reconstruction NLL of the low-precision HIP
training path against an fp32 reference at equal steps.

Every arm trains the same model (same init seed) on the same synthetic
stroke-5 corpus with the same batch order, then evaluates the held-out recon
NLL (``r_cost``: shape + pen terms, no dropout, fixed reparameterisation
noise) every ``--eval-every`` steps. Arms:

* ``hip-bf16``  -- the benchmarked path (HIP kernels, bf16 MFMA operands,
  fp32 state/accumulation, one HIP graph per step);
* ``hip-fp32``  -- HIP kernels with fp32 operands;
* ``torch-fp32`` -- the PyTorch oracle (fp32 autograd recurrences; slow: use
  on the small config).

One JSON line per arm: the NLL curve, the final NLL and its relative gap to
the first fp32 arm. Synthetic data only (no dataset in this environment):
this pins precision parity, not the QuickDraw literature number.

Usage: python scripts/converge.py --config vae_small --steps 2000 \
           --arms hip-bf16,torch-fp32 --out profiles/r2_converge_small.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def run_arm(arm: str, args, seed: int = 0) -> dict:
    import torch
    from sketch_rnn_amd import ops
    from sketch_rnn_amd.config import PRESETS
    from sketch_rnn_amd.data.dataset import StrokeDataset
    from sketch_rnn_amd.data.synthetic import synthetic_corpus
    from sketch_rnn_amd.train.trainer import VAETrainer

    backend, dtype = arm.split("-")
    ops.set_backend(backend)
    cfg = PRESETS[args.config].replace(batch_size=args.batch, max_seq_len=args.seq_len, save_every=0, seed=seed)
    strokes, labels = synthetic_corpus(args.sketches, seed=1234, max_len=args.seq_len,
                                       n_classes=max(cfg.num_classes, 1))
    n_test = max(args.batch, len(strokes) // 10)
    train = StrokeDataset(strokes[n_test:], args.batch, args.seq_len, random_scale_factor=cfg.random_scale_factor,
                          augment_stroke_prob=cfg.augment_stroke_prob, labels=labels[n_test:], seed=7 + 101 * seed)
    scale = train.normalize()
    test = StrokeDataset(strokes[:n_test], args.batch, args.seq_len, labels=labels[:n_test], seed=8)
    test.normalize(scale)
    torch.manual_seed(seed)
    trainer = VAETrainer(cfg, train, None, test, device="cuda", save_dir="/tmp/skr_converge",
                         use_graph=(backend == "hip"), log=lambda s: None, compute_dtype=dtype)
    trainer.seed.fill_(1000003 * seed)       # dropout / reparameterisation noise stream of this seed
    curve = []
    t0 = time.perf_counter()
    print("%s seed %d: training %d steps" % (arm, seed, args.steps), file=sys.stderr, flush=True)
    for step in range(1, args.steps + 1):
        out = trainer.train_step(*trainer.batch_to_device(train.random_batch()))
        if step % 50 == 0:   # heartbeat (the GPU runner kills a silent run)
            print("%s seed %d step %d" % (arm, seed, step), file=sys.stderr, flush=True)
        if step % args.eval_every == 0 or step == args.steps:
            ev = trainer.evaluate(test)
            curve.append({"step": step, "test_recon_nll": round(ev["r_cost"], 5), "test_kl": round(ev["kl_cost"], 5),
                          "train_cost": round(float(out["cost"]), 5),
                          "wall_s": round(time.perf_counter() - t0, 1)})
            print("%s seed %d step %d: test recon NLL %.4f (train cost %.4f, %.0f s)"
                  % (arm, seed, step, ev["r_cost"], float(out["cost"]), time.perf_counter() - t0),
                  file=sys.stderr, flush=True)
    return {"arm": arm, "seed": seed, "commit": args.commit, "config": args.config, "steps": args.steps, "batch": args.batch, "seq_len": args.seq_len,
            "curve": curve, "final_test_recon_nll": curve[-1]["test_recon_nll"],
            "skipped_steps": trainer.opt.skipped_steps()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="vae_small")
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--eval-every", type=int, default=250)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--seq-len", type=int, default=250)
    ap.add_argument("--sketches", type=int, default=5000)
    ap.add_argument("--arms", default="hip-bf16,hip-fp32")
    ap.add_argument("--seeds", default="0", help="comma list: init, data-order and noise seed of each run")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    # the tree's identity, taken by the run itself: git HEAD + dirty flag (or
    # TREE_COMMIT on a box without .git) and a recomputable source hash
    from sketch_rnn_amd.utils.provenance import tree_identity
    args.commit = tree_identity()
    import numpy as np
    seeds = [int(x) for x in args.seeds.split(",")]
    arms = args.arms.split(",")
    res = []
    for sd in seeds:
        for a in arms:
            r = run_arm(a, args, sd)
            res.append(r)
            print(json.dumps(r), flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(json.dumps(r) + "\n")
    # mean +- std of the final test recon NLL per arm over the seeds
    summ = {"summary": True, "commit": args.commit, "config": args.config, "steps": args.steps, "seeds": seeds, "arms": {}}
    for a in arms:
        v = np.array([r["final_test_recon_nll"] for r in res if r["arm"] == a])
        summ["arms"][a] = {"mean": round(float(v.mean()), 5), "std": round(float(v.std(ddof=1)) if len(v) > 1 else 0.0, 5),
                           "finals": [float(x) for x in v]}
    ref = next((a for a in arms if a.endswith("fp32")), None)
    if ref is not None:
        m0 = summ["arms"][ref]["mean"]
        for a in arms:
            if a != ref:
                d = summ["arms"][a]["mean"] - m0
                summ["arms"][a]["rel_gap_vs_%s" % ref] = round(d / abs(m0), 5)
                summ["arms"][a]["gap_in_%s_std" % ref] = round(d / max(summ["arms"][ref]["std"], 1e-12), 3)
    print(json.dumps(summ), flush=True)
    if args.out:
        with open(args.out, "a") as f:
            f.write(json.dumps(summ) + "\n")


if __name__ == "__main__":
    main()
