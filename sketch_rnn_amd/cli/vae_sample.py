"""``python -m sketch_rnn_amd.cli.vae_sample`` -- generate from a trained VAE.

Modes: ``random`` (z ~ N(0, I), or the unconditional decoder), ``class``
(class-conditional z for ``--label``), ``interpolate`` (spherical
interpolation between two random latents). Writes a stroke-3 SVG grid.
``--device_sampler`` decodes the whole grid in parallel through the
HIP-graph decoder.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np


def slerp(p0, p1, t):
    p0, p1 = np.asarray(p0, np.float64), np.asarray(p1, np.float64)
    omega = np.arccos(np.clip(np.dot(p0 / np.linalg.norm(p0), p1 / np.linalg.norm(p1)), -1, 1))
    so = np.sin(omega)
    if so < 1e-8:
        return (1.0 - t) * p0 + t * p1
    return np.sin((1.0 - t) * omega) / so * p0 + np.sin(t * omega) / so * p1


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    p.add_argument("--save_dir", default="save/vae")
    p.add_argument("--out", default="vae_samples.svg")
    p.add_argument("--mode", choices=["random", "class", "interpolate"], default="random")
    p.add_argument("--n", type=int, default=10)
    p.add_argument("--label", type=int, default=0)
    p.add_argument("--temperature", type=float, default=0.5)
    p.add_argument("--greedy", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--device", default=None)
    p.add_argument("--device_sampler", action="store_true")
    p.add_argument("--fp8", action="store_true",
                   help="device sampler: h W_h of the HyperLSTM decoder as an MX-fp8 GEMM (BASELINE config 5; "
                        "pays at >= 1024 sketches per call)")
    a = p.parse_args(argv)
    import torch
    from ..ckpt import checkpoint as ckpt
    from ..config import load_json
    from ..data.strokes import to_normal_strokes
    from ..models.vae import SketchVAE
    from ..render.svg import grid_strokes3
    from ..sample.sampler import GraphDecoder, sample_vae
    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    cfg = load_json(os.path.join(a.save_dir, "config.json"))
    model = SketchVAE(cfg).to(device)
    path = ckpt.latest_checkpoint(a.save_dir)
    if path:
        ckpt.load_checkpoint(path, model)
    model.eval()
    rng = np.random.RandomState(a.seed)
    zs = rng.randn(a.n, cfg.z_size)
    if a.mode == "interpolate":
        z0, z1 = rng.randn(cfg.z_size), rng.randn(cfg.z_size)
        zs = np.stack([slerp(z0, z1, t) for t in np.linspace(0, 1, a.n)])
    labels = np.full(a.n, a.label if a.mode == "class" else 0)
    sketches = []
    if a.device_sampler and device.startswith("cuda"):
        dec = GraphDecoder(model, a.n, cfg.max_seq_len, a.temperature, a.greedy, fp8=a.fp8)
        s, _ = dec.run(seed=a.seed, z=torch.as_tensor(zs, dtype=torch.float32, device=device),
                       labels=torch.as_tensor(labels, device=device))
        sketches = [to_normal_strokes(x) for x in s.cpu().numpy()]
    else:
        for k in range(a.n):
            z = torch.as_tensor(zs[k:k + 1], dtype=torch.float32, device=device)
            s5, _ = sample_vae(model, cfg.max_seq_len, a.temperature, a.greedy, z=z, label=int(labels[k]), rng=rng)
            sketches.append(to_normal_strokes(s5))
    grid_strokes3(sketches, a.out)
    print("wrote %s (%d sketches)" % (a.out, len(sketches)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
