#!/usr/bin/env python3
"""BASELINE config 5: fp8 gate GEMM in the HyperLSTM decode step (dec 2048),
temperature-sampled generation under HIP graphs -- quality and speed
against the same decoder with bf16 GEMMs.

1. Train the model ``--train-steps`` steps (bf16, synthetic sketches; a
   random-init decoder ends its sketches after a few strokes).
2. Quality: teacher-forced reconstruction NLL of the held-out split through
   the step decoder (``sample/hyper_step.py`` four/five-launch stroke, the
   path generation runs), z = the encoder mean; MDN loss in fp32 torch
   (``models/mdn.py``, magenta mode, pen term on valid steps). bf16 vs fp8
   ``h W_h`` on identical weights and inputs.
3. Speed: ``GraphDecoder`` (chunked HIP graphs, all-done exit) at each
   ``--batches`` size, bf16 vs fp8, the same seeds: valid strokes/s (sum of
   the sketch lengths / wall) and decode positions/s.

One JSON line per measurement, then a summary line."""
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
    ap.add_argument("--train-steps", type=int, default=300)
    ap.add_argument("--seq-len", type=int, default=250)
    ap.add_argument("--eval-batches", type=int, default=4)
    ap.add_argument("--batches", default="128,1024")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--temperature", type=float, default=0.5)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import torch
    from sketch_rnn_amd import ops
    from sketch_rnn_amd.config import PRESETS
    from sketch_rnn_amd.data.dataset import StrokeDataset
    from sketch_rnn_amd.data.synthetic import synthetic_corpus
    from sketch_rnn_amd.models.mdn import mdn_loss_torch
    from sketch_rnn_amd.sample.hyper_step import HyperStepDecoder
    from sketch_rnn_amd.sample.sampler import GraphDecoder
    from sketch_rnn_amd.train.trainer import VAETrainer
    from sketch_rnn_amd.utils.provenance import tree_identity

    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    dev = torch.device("cuda")
    cfg = PRESETS[a.config].replace(max_seq_len=a.seq_len, batch_size=100, save_every=0, seed=a.seed)
    strokes, labels = synthetic_corpus(4000, seed=1234 + a.seed, max_len=a.seq_len, n_classes=max(cfg.num_classes, 1))
    n_test = 100 * a.eval_batches
    train = StrokeDataset(strokes[n_test:], 100, a.seq_len, labels=labels[n_test:], seed=7 + a.seed)
    scale = train.normalize()
    test = StrokeDataset(strokes[:n_test], 100, a.seq_len, labels=labels[:n_test], seed=8)
    test.normalize(scale)
    tr = VAETrainer(cfg, train, None, test, device="cuda", save_dir="/tmp/skr_fp8_eval", log=lambda s: None,
                    compute_dtype="bf16")
    t0 = time.perf_counter()
    for _ in range(a.train_steps):
        out = tr.train_step(*tr.batch_to_device(train.random_batch()))
    torch.cuda.synchronize()
    m = tr.model.eval()
    ident = tree_identity()
    print(json.dumps({"phase": "train", "config": a.config, "steps": a.train_steps, "train_cost": float(out["cost"]),
                      "wall_s": round(time.perf_counter() - t0, 1), "tree": ident}), flush=True)

    # ---- quality: teacher-forced recon NLL through the step decoder
    nll = {}
    with torch.no_grad():
        for arm in ("bf16", "fp8"):
            tot = n = 0.0
            for b in range(test.num_batches):
                s, l, c = tr.batch_to_device(test.get_batch(b))
                B, N = s.shape[0], s.shape[1] - 1
                mu, _ = m.encode(s, l)
                zc = m.condition(mu, c if cfg.num_classes > 0 else None, B, dev)
                st = HyperStepDecoder(m, B, dev, fp8=(arm == "fp8"))
                assert st.fused and st.fp8 == (arm == "fp8")
                st.begin(zc, m.initial_state(zc, B, dev))
                zs = []
                for t in range(N):
                    st.X.copy_(s[:, t])
                    st.step_fused(t, None)
                    st.head()
                    zs.append(st.ZS.sum(0)[:, :cfg.n_out] + st._w["bo"][:cfg.n_out])
                z = torch.stack(zs)                                    # [N, B, nout]
                tgt = s[:, 1:].transpose(0, 1)                         # [N, B, 5]
                r, _, _ = mdn_loss_torch(z, tgt, cfg.num_mixture, mode="magenta", is_training=False)
                tot += float(r)
                n += 1
            nll[arm] = tot / n
            print(json.dumps({"phase": "quality", "arm": arm, "teacher_forced_recon_nll": round(nll[arm], 5),
                              "batches": int(n)}), flush=True)
    rel = (nll["fp8"] - nll["bf16"]) / abs(nll["bf16"])

    # ---- speed: graph decode, bf16 vs fp8, same seeds (alternating arms)
    speed = {}
    for B in [int(x) for x in a.batches.split(",")]:
        decs = {arm: GraphDecoder(m, B, a.seq_len, a.temperature, fp8=(arm == "fp8")) for arm in ("bf16", "fp8")}
        for arm, d in decs.items():
            d.run(seed=0)                                              # capture
        torch.cuda.synchronize()
        for arm in ("bf16", "fp8", "bf16", "fp8"):
            d = decs[arm]
            tl = tp = 0
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for r in range(a.reps):
                _, lens = d.run(seed=r + 1)
                tl += int(lens.sum())
                tp += B * d.steps_run
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            rec = {"phase": "speed", "arm": arm, "batch": B, "valid_strokes_per_s": round(tl / wall, 1),
                   "decode_positions_per_s": round(tp / wall, 1), "mean_len": tl / B / a.reps,
                   "ms_per_decode_step": round(1000 * wall / (tp / B), 4)}
            speed.setdefault((B, arm), []).append(rec["decode_positions_per_s"])
            print(json.dumps(rec), flush=True)
    summ = {"summary": True, "config": a.config, "train_steps": a.train_steps, "tree": ident,
            "teacher_forced_recon_nll": nll, "fp8_vs_bf16_nll_rel": round(rel, 5),
            "decode_speedup_fp8_vs_bf16": {str(B): round(max(speed[(B, "fp8")]) / max(speed[(B, "bf16")]), 3)
                                           for B in sorted({k[0] for k in speed})}}
    print(json.dumps(summ), flush=True)


if __name__ == "__main__":
    main()
