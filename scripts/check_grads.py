#!/usr/bin/env python3
"""Per-parameter gradient check of a VAE preset: the HIP path (bf16 or fp32
operands) against the PyTorch fp32 path on the same batch, same seeds.
Prints the loss of both and, per parameter, the relative L2 error of the
gradient (|g_hip - g_ref| / |g_ref|) -- a diagnostics tool for kernel
changes whose unit tests pass at small shapes.
usage: python scripts/check_grads.py [--config vae_large] [--dtype bf16] [--seq-len 64]"""
import argparse
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="vae_large")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--batch", type=int, default=100)
    ap.add_argument("--seq-len", type=int, default=64)
    ap.add_argument("--perturb", type=float, default=0.02, help="noise added to every weight (moves off the "
                    "init, where the hyper-network gradients are exactly zero)")
    a = ap.parse_args()
    from sketch_rnn_amd import ops
    from sketch_rnn_amd.config import PRESETS
    from sketch_rnn_amd.data.dataset import StrokeDataset
    from sketch_rnn_amd.data.synthetic import synthetic_corpus
    from sketch_rnn_amd.models.vae import SketchVAE
    dev = torch.device("cuda")
    cfg = PRESETS[a.config].replace(batch_size=a.batch, max_seq_len=a.seq_len)
    strokes, labels = synthetic_corpus(400, seed=3, max_len=a.seq_len, n_classes=max(cfg.num_classes, 1))
    ds = StrokeDataset(strokes, a.batch, a.seq_len, labels=labels, seed=1)
    ds.normalize()
    s, l, c = ds.random_batch()
    s, l = torch.as_tensor(s, device=dev), torch.as_tensor(l, device=dev)
    c = torch.as_tensor(c, device=dev) if cfg.num_classes > 0 else None
    model = SketchVAE(cfg).to(dev)
    with torch.no_grad():
        g = torch.Generator(device=dev).manual_seed(0)
        for p in model.parameters():
            p.add_(torch.randn(p.shape, device=dev, generator=g) * a.perturb)
    res = {}
    for name, backend, dt in (("hip", "hip", a.dtype), ("ref", "torch", "fp32")):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        model.zero_grad()
        out = model.loss(s, l, c, kl_weight=0.5, seed=7)
        out["cost"].backward()
        torch.cuda.synchronize()
        res[name] = (float(out["cost"]), {n: p.grad.detach().clone() for n, p in model.named_parameters()
                                          if p.grad is not None})
    print("cost hip %.6f ref %.6f" % (res["hip"][0], res["ref"][0]))
    worst = 0.0
    for n, g in res["ref"][1].items():
        gh = res["hip"][1].get(n)
        if gh is None:
            print("%-40s missing in hip" % n)
            continue
        rel = ((gh - g).norm() / g.norm().clamp_min(1e-30)).item()
        worst = max(worst, rel)
        print("%-40s rel %.3e  |g| %.3e" % (n, rel, g.norm().item()))
    print("worst rel err %.3e" % worst)


if __name__ == "__main__":
    main()
