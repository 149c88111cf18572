#!/usr/bin/env python3
"""Which parameter gradients of a training step are NOT produced in their
optimizer-arena slot (and so are copied by gather_grads' multi-tensor copy):
one eager forward + backward of the preset on synthetic data, then one JSON
line per copied gradient and a total. usage: grad_copies.py [preset]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.config import PRESETS  # noqa: E402
from sketch_rnn_amd.data.dataset import StrokeDataset  # noqa: E402
from sketch_rnn_amd.data.synthetic import synthetic_corpus  # noqa: E402
from sketch_rnn_amd.train.trainer import VAETrainer  # noqa: E402


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "vae_large"
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    ops.set_backend("hip" if dev == "cuda" else "torch")
    cfg = PRESETS[preset].replace(save_every=0)
    strokes, labels = synthetic_corpus(400, seed=1234, max_len=cfg.max_seq_len, n_classes=max(cfg.num_classes, 1))
    train = StrokeDataset(strokes, cfg.batch_size, cfg.max_seq_len, labels=labels, seed=7)
    train.normalize()
    tr = VAETrainer(cfg, train, None, None, device=dev, save_dir="/tmp/skr_gc", use_graph=False,
                    log=lambda s: None, compute_dtype="bf16")
    s, L, lab = tr.batch_to_device(train.random_batch(0, 1))
    opt = tr.opt
    opt.zero_grad(set_to_none=True)
    out = tr.model.loss(s, L, lab if cfg.num_classes > 0 else None, kl_weight=tr.kl_w, train=True, seed=tr.seed)
    out["cost"].backward()
    names = {id(p): n for n, p in tr.model.named_parameters()}
    total = 0
    for p, o in zip(opt.params, opt.offsets):
        view = opt.grad[o:o + p.numel()]
        g = p.grad
        if g is None or g.data_ptr() != view.data_ptr():
            nbytes = 0 if g is None else g.numel() * g.element_size()
            total += nbytes
            print(json.dumps({"param": names.get(id(p), "?"), "shape": list(p.shape),
                              "grad": "none (zero-filled)" if g is None else "copied", "bytes": nbytes}))
    print(json.dumps({"preset": preset, "copied_bytes": total}))


if __name__ == "__main__":
    main()
