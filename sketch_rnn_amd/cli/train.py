"""``python -m sketch_rnn_amd.cli.train`` -- reference training CLI (``train.py:12-45``).

Same flags and defaults as the reference; additions: ``--data_dir``,
``--save_root``, ``--device``, ``--seed``, ``--resume``, ``--max_batches``,
``--synthetic N`` (train on N synthetic sketches when no dataset exists),
``--metrics`` (JSONL log) and ``--no_graph``.
"""
from __future__ import annotations

import argparse
import os
import sys


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="train the sketch-rnn MDN-RNN (reference model)")
    p.add_argument("--rnn_size", type=int, default=256, help="size of RNN hidden state")
    p.add_argument("--num_layers", type=int, default=2, help="number of layers in the RNN")
    p.add_argument("--model", type=str, default="lstm", help="rnn, gru, or lstm")
    p.add_argument("--batch_size", type=int, default=100, help="minibatch size")
    p.add_argument("--seq_length", type=int, default=300, help="RNN sequence length")
    p.add_argument("--num_epochs", type=int, default=500, help="number of epochs")
    p.add_argument("--save_every", type=int, default=250, help="save frequency")
    p.add_argument("--grad_clip", type=float, default=5.0, help="clip gradients at this value")
    p.add_argument("--learning_rate", type=float, default=0.005, help="learning rate")
    p.add_argument("--decay_rate", type=float, default=0.99, help="decay rate after each epoch (adam is used)")
    p.add_argument("--num_mixture", type=int, default=24, help="number of gaussian mixtures")
    p.add_argument("--data_scale", type=float, default=15.0, help="factor to scale raw data down by")
    p.add_argument("--keep_prob", type=float, default=0.8, help="dropout keep probability")
    p.add_argument("--stroke_importance_factor", type=float, default=200.0,
                   help="relative importance of pen status over mdn coordinate accuracy")
    p.add_argument("--dataset_name", type=str, default="kanji", help="name of directory containing training data")
    # framework additions
    p.add_argument("--data_dir", type=str, default="./data")
    p.add_argument("--save_root", type=str, default="save")
    p.add_argument("--device", type=str, default="cuda" if _has_cuda() else "cpu")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--max_batches", type=int, default=None)
    p.add_argument("--synthetic", type=int, default=0, help="use N synthetic sketches instead of a dataset")
    p.add_argument("--metrics", type=str, default=None)
    p.add_argument("--no_graph", action="store_true")
    p.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    return p


def _has_cuda() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    from .. import ops
    from ..config import RefConfig
    from ..data.loader import SketchLoader
    from ..train.trainer import ReferenceTrainer
    cfg = RefConfig(**{k: getattr(args, k) for k in RefConfig.__dataclass_fields__ if hasattr(args, k)})
    ops.set_compute_dtype(args.dtype)
    sketches = None
    if args.synthetic:
        from ..data.synthetic import synthetic_reference_corpus
        sketches = synthetic_reference_corpus(args.synthetic, seed=args.seed)
    loader = SketchLoader(cfg.batch_size, cfg.seq_length, cfg.data_scale, cfg.dataset_name, data_dir=args.data_dir,
                          sketches=sketches, seed=args.seed)
    tr = ReferenceTrainer(cfg, loader, device=args.device, save_root=args.save_root,
                          use_graph=False if args.no_graph else None, metrics_path=args.metrics)
    if args.resume:
        tr.resume()
    tr.train(max_batches=args.max_batches)
    return 0


if __name__ == "__main__":
    sys.exit(main())
