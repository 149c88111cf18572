#!/usr/bin/env python3
"""Reference-model training throughput (SURVEY §7.3 "minimum end-to-end
slice"): the reference's checkpointed config -- 2 x 256 LSTM, M = 24,
B = 100, T = 300, keep 0.8, TF Adam + global clip 5, eoc state reset,
TBPTT state carry -- one full training step per iteration, on synthetic
packed kanji-like data.

Comparators on the same GPU:
  * ``--backend torch``: the same model with PyTorch ops for the recurrence;
  * ``--cudnn``: a "reference-equivalent" PyTorch model on ``torch.nn.LSTM``
    (MIOpen) + the same MDN loss and optimizer -- without the eoc reset,
    which nn.LSTM cannot express, so it does strictly less work.

Prints one JSON line.
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--cudnn", action="store_true")
    ap.add_argument("--model", default="lstm")
    a = ap.parse_args()
    import torch
    from sketch_rnn_amd import ops
    from sketch_rnn_amd.config import RefConfig
    from sketch_rnn_amd.data.loader import SketchLoader
    from sketch_rnn_amd.data.synthetic import synthetic_reference_corpus
    from sketch_rnn_amd.train.trainer import ReferenceTrainer, _to_device

    ops.set_backend(a.backend)
    ops.set_compute_dtype(a.dtype)
    cfg = RefConfig(model=a.model)
    loader = SketchLoader(cfg.batch_size, cfg.seq_length, cfg.data_scale, sketches=synthetic_reference_corpus(4000, seed=0),
                          seed=0)
    dev = "cuda"
    batches = [tuple(_to_device(v, dev) for v in loader.next_batch()) for _ in range(4)]
    if a.cudnn:
        from sketch_rnn_amd.models.mdn import mdn_loss_torch
        from sketch_rnn_amd.train.optim import FlatAdam
        lstm = torch.nn.LSTM(5, cfg.rnn_size, cfg.num_layers, batch_first=True).to(dev)
        head = torch.nn.Linear(cfg.rnn_size, cfg.n_out).to(dev)
        params = list(lstm.parameters()) + list(head.parameters())
        opt = FlatAdam(params, lr=cfg.learning_rate, eps=cfg.adam_eps, clip_mode="global_norm", clip=cfg.grad_clip)
        lstm.flatten_parameters()
        state = None

        amp = a.dtype == "bf16"   # bf16 comparator: MIOpen LSTM + head under autocast, fp32 master weights

        def step(x, y):
            nonlocal state
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                out, st = lstm(x, state)
                out = torch.nn.functional.dropout(out, 1 - cfg.keep_prob)
                z = head(out.reshape(-1, cfg.rnn_size))
            cost = mdn_loss_torch(z.float(), y.reshape(-1, 5), cfg.num_mixture, mode="reference")[0]
            cost.backward()
            opt.step()
            state = tuple(s.detach().float() for s in st)
            return cost
    else:
        tr = ReferenceTrainer(cfg, loader, device=dev, log=lambda s: None)

        def step(x, y):
            return tr.train_step(x, y)["cost"]
    for i in range(a.warmup):
        step(*batches[i % 4])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        c = step(*batches[i % 4])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({"metric": "reference model train strokes/s", "model": "%dx%d %s M=%d B=%d T=%d" % (
        cfg.num_layers, cfg.rnn_size, cfg.model, cfg.num_mixture, cfg.batch_size, cfg.seq_length),
        "impl": "nn.LSTM(MIOpen) comparator" if a.cudnn else "sketch_rnn_amd backend=%s" % ops.get_backend(),
        "dtype": a.dtype, "ms_per_step": round(1000 * dt, 3),
        "strokes_per_s": round(cfg.batch_size * cfg.seq_length / dt, 1), "cost": round(float(c), 4)}), flush=True)


if __name__ == "__main__":
    main()
