"""``python -m sketch_rnn_amd.cli.vae_train`` -- seq2seq VAE training.

Every :class:`~sketch_rnn_amd.config.VAEConfig` field is a flag
(``--dec_model hyper --dec_rnn_size 2048 ...``) or comes from ``--preset``
(``plumbing | vae_small | vae_large | vae_classcond | vae_layernorm``).
Data: ``--data path.skpack.npz`` (see ``data.quickdraw``) or
``--synthetic N``. Offsets are normalised by the training set's standard
deviation (stored in the checkpoint config as ``scale_factor``).

Multi-GPU: ``python -m torch.distributed.run --nproc-per-node 8
--master-addr 127.0.0.1 -m sketch_rnn_amd.cli.vae_train ...`` (one rank per
GPU, RCCL all-reduce of the flat gradient arena).
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys


def build_parser():
    from ..config import VAEConfig
    p = argparse.ArgumentParser(description="train the sketch-rnn seq2seq VAE")
    p.add_argument("--preset", default=None)
    for f in dataclasses.fields(VAEConfig):
        if f.name == "kind":
            continue
        t = f.type if not isinstance(f.type, str) else {"int": int, "float": float, "str": str, "bool": bool}[f.type]
        if t is bool:
            p.add_argument("--" + f.name, type=lambda s: s.lower() in ("1", "true", "yes"), default=None)
        else:
            p.add_argument("--" + f.name, type=t, default=None)
    p.add_argument("--data", default=None, help="sketch pack (.npz) with train/valid/test splits")
    p.add_argument("--synthetic", type=int, default=0)
    p.add_argument("--save_dir", default="save/vae")
    p.add_argument("--device", default=None)
    p.add_argument("--dtype", choices=["fp32", "bf16"], default="bf16")
    p.add_argument("--eval_every", type=int, default=0)
    p.add_argument("--log_every", type=int, default=20)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--metrics", default=None)
    p.add_argument("--no_graph", action="store_true")
    return p


def make_datasets(cfg, data_path, synthetic, rank=0):
    from ..data.dataset import StrokeDataset
    if data_path:
        from ..data.quickdraw import load_pack
        splits = load_pack(data_path)
    else:
        from ..data.synthetic import synthetic_corpus
        n = synthetic or 2000
        s, l = synthetic_corpus(n, seed=cfg.seed, max_len=cfg.max_seq_len, n_classes=max(cfg.num_classes, 1))
        k = max(n // 10, cfg.batch_size)
        splits = {"train": (s[2 * k:], l[2 * k:]), "valid": (s[:k], l[:k]), "test": (s[k:2 * k], l[k:2 * k])}
    train = StrokeDataset(splits["train"][0], cfg.batch_size, cfg.max_seq_len, random_scale_factor=cfg.random_scale_factor,
                          augment_stroke_prob=cfg.augment_stroke_prob, labels=splits["train"][1], seed=cfg.seed, rank=rank)
    scale = train.normalize()
    out = [train]
    for name in ("valid", "test"):
        if name in splits:
            ds = StrokeDataset(splits[name][0], cfg.batch_size, cfg.max_seq_len, labels=splits[name][1])
            ds.normalize(scale)
            out.append(ds)
        else:
            out.append(None)
    return out, scale


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    import torch
    from ..config import PRESETS, VAEConfig
    from ..parallel import dp
    from ..train.trainer import VAETrainer
    cfg = PRESETS[a.preset] if a.preset else VAEConfig()
    over = {f.name: getattr(a, f.name) for f in dataclasses.fields(VAEConfig)
            if f.name != "kind" and getattr(a, f.name, None) is not None}
    cfg = dataclasses.replace(cfg, **over)
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = a.device or ("cuda:%d" % local_rank if torch.cuda.is_available() else "cpu")
    if device.startswith("cuda"):
        torch.cuda.set_device(torch.device(device))
    dp.init_from_env(device=device)
    (train, valid, test), scale = make_datasets(cfg, a.data, a.synthetic, dp.rank())
    tr = VAETrainer(cfg, train, valid, test, device=device, save_dir=a.save_dir,
                    use_graph=False if a.no_graph else None, metrics_path=a.metrics, compute_dtype=a.dtype)
    if dp.rank() == 0:
        os.makedirs(a.save_dir, exist_ok=True)
        with open(os.path.join(a.save_dir, "data.json"), "w") as f:
            json.dump({"scale_factor": scale}, f)
    if a.resume:
        tr.resume()
    tr.train(eval_every=a.eval_every, log_every=a.log_every)
    if test is not None and test.num_batches > 0:
        ev = tr.evaluate(test)
        if dp.rank() == 0:
            print("test: cost %.4f recon NLL %.4f kl %.4f" % (ev["cost"], ev["r_cost"], ev["kl_cost"]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
