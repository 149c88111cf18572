#!/usr/bin/env python3
"""Library comparator for the LSTM-decoder VAE presets (VERDICT r1 "What's
weak" 2): the same seq2seq VAE written on ``torch.nn.LSTM`` (MIOpen) --
bidirectional encoder, z from (mu, sigma), decoder initial state
``tanh(z W + b)``, decoder input ``[stroke-5 | z]``, linear MDN head, the
magenta MDN loss + KL, TF-style Adam with per-element gradient clipping --
one full training step per iteration on the same synthetic batches as
``bench.py``, optionally under bf16 autocast (fp32 master weights).

Differences, all of which make the comparator do LESS work than
``bench.py``: no recurrent dropout (MIOpen has none), the encoder's backward
direction runs over the padded sequence instead of each sketch's reversed
prefix, and no HIP graph. LayerNorm / HyperLSTM decoders have no MIOpen
kernel, so only ``dec_model == "lstm"`` presets are accepted.

Prints one JSON line (``ms_per_step`` and padded ``positions_per_s`` like
``bench.py``).
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
    ap.add_argument("--config", default="vae_small")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--seq-len", type=int, default=250)
    ap.add_argument("--dtype", default="bf16", choices=["fp32", "bf16"])
    a = ap.parse_args()
    import torch
    import torch.nn as nn
    from sketch_rnn_amd.config import PRESETS
    from sketch_rnn_amd.data.dataset import StrokeDataset
    from sketch_rnn_amd.data.synthetic import synthetic_corpus
    from sketch_rnn_amd.models.mdn import mdn_loss_torch
    from sketch_rnn_amd.train.optim import FlatAdam

    cfg = PRESETS[a.config].replace(batch_size=a.batch, max_seq_len=a.seq_len)
    if cfg.dec_model != "lstm" or cfg.enc_model != "lstm":
        raise SystemExit("MIOpen comparator: plain LSTM encoder/decoder presets only (got %s/%s)"
                         % (cfg.enc_model, cfg.dec_model))
    dev = "cuda"
    strokes, labels = synthetic_corpus(2000, seed=1234, max_len=a.seq_len)
    ds = StrokeDataset(strokes, a.batch, a.seq_len, random_scale_factor=cfg.random_scale_factor,
                       augment_stroke_prob=cfg.augment_stroke_prob, labels=labels, seed=7)
    ds.normalize()

    class VAE(nn.Module):
        def __init__(self):
            super().__init__()
            E, H, Z = cfg.enc_rnn_size, cfg.dec_rnn_size, cfg.z_size
            self.enc = nn.LSTM(5, E, batch_first=False, bidirectional=True)
            self.mu = nn.Linear(2 * E, Z)
            self.sig = nn.Linear(2 * E, Z)
            self.init = nn.Linear(Z, 2 * H)
            self.dec = nn.LSTM(5 + Z, H, batch_first=False)
            self.head = nn.Linear(H, cfg.n_out)

        def forward(self, s, lengths):
            T = s.shape[1] - 1
            x = s[:, 1:].transpose(0, 1)                       # [T, B, 5]
            out, _ = self.enc(x)
            B = x.shape[1]
            E = cfg.enc_rnn_size
            idx = (lengths - 1).clamp(min=0).view(1, B, 1).expand(1, B, 2 * E)
            last = torch.gather(out, 0, idx).squeeze(0)
            mu, presig = self.mu(last), self.sig(last)
            z = mu + torch.exp(presig / 2) * torch.randn_like(mu)
            h0, c0 = torch.tanh(self.init(z)).chunk(2, -1)
            xin = torch.cat([s[:, :T].transpose(0, 1), z.unsqueeze(0).expand(T, B, z.shape[-1])], -1)
            dout, _ = self.dec(xin, (h0.unsqueeze(0).contiguous(), c0.unsqueeze(0).contiguous()))
            zh = self.head(dout.reshape(-1, cfg.dec_rnn_size))
            kl = -0.5 * torch.mean(1 + presig - mu * mu - torch.exp(presig))
            return zh, kl.float().clamp(min=cfg.kl_tolerance)

    model = VAE().to(dev)
    model.enc.flatten_parameters()
    model.dec.flatten_parameters()
    opt = FlatAdam(model.parameters(), lr=cfg.learning_rate, eps=cfg.adam_eps, clip_mode="value", clip=cfg.grad_clip)
    amp = a.dtype == "bf16"

    def to_dev(b):
        s, l, _ = b
        return torch.as_tensor(s, device=dev, dtype=torch.float32), torch.as_tensor(l, device=dev, dtype=torch.int64)

    batches = [to_dev(ds.random_batch()) for _ in range(4)]
    valid = [float(b[1].sum()) for b in batches]

    def step(s, lengths):
        opt.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            zh, kl = model(s, lengths)
        target = s[:, 1:].transpose(0, 1).reshape(-1, 5)
        r = mdn_loss_torch(zh.float(), target, cfg.num_mixture, mode="magenta")[0]
        cost = r + cfg.kl_weight * kl
        cost.backward()
        opt.step()
        return cost

    for i in range(a.warmup):
        step(*batches[i % 4])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        c = step(*batches[i % 4])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(json.dumps({
        "metric": "VAE train strokes/s, nn.LSTM (MIOpen) comparator", "config": a.config,
        "model": "enc %d biLSTM / dec %d LSTM, z %d, M=%d" % (cfg.enc_rnn_size, cfg.dec_rnn_size, cfg.z_size,
                                                             cfg.num_mixture),
        "dtype": a.dtype, "batch": a.batch, "seq_len": a.seq_len, "ms_per_step": round(1000 * dt, 3),
        "positions_per_s": round(a.batch * a.seq_len / dt, 1),
        "valid_strokes_per_s": round(sum(valid[i % 4] for i in range(a.steps)) / (dt * a.steps), 1),
        "cost": round(float(c), 4)}), flush=True)


if __name__ == "__main__":
    main()
