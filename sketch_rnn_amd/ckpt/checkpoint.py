"""Checkpoint format (reference capability R16).

Directory contract kept from the reference (``train.py:54-75``,
``save/kanji/checkpoint``)::

    save/<dataset>/
        config.json                      # typed config (RefConfig / VAEConfig)
        checkpoint                       # text index, TF style:
                                         #   model_checkpoint_path: "model.ckpt-N"
                                         #   all_model_checkpoint_paths: "model.ckpt-..."
        model.ckpt-N.safetensors         # tensors + JSON metadata

Tensors: ``model/<param>`` (fp32 weights), ``optim/m``, ``optim/v``,
``optim/scalars`` (Adam moments + [lr, t, grad_norm, clip_scale]),
``state/<k>`` (carried RNN state for reference-mode TBPTT). Metadata
(``__metadata__``): step, epoch, loader cursor, RNG states -> true resume
(the reference's resume is commented out, ``train.py:66-70``).
safetensors never executes code on load.
"""
from __future__ import annotations

import json
import os
import re
from typing import Any, Dict, Optional

import torch
from safetensors.torch import load_file, save_file

INDEX = "checkpoint"
_RE = re.compile(r'^(\w+):\s*"(.*)"\s*$')


def _read_index(save_dir: str):
    p = os.path.join(save_dir, INDEX)
    if not os.path.exists(p):
        return None, []
    latest, allp = None, []
    with open(p) as f:
        for line in f:
            m = _RE.match(line.strip())
            if not m:
                continue
            if m.group(1) == "model_checkpoint_path":
                latest = m.group(2)
            elif m.group(1) == "all_model_checkpoint_paths":
                allp.append(m.group(2))
    return latest, allp


def _write_index(save_dir: str, latest: str, allp):
    tmp = os.path.join(save_dir, INDEX + ".tmp")
    with open(tmp, "w") as f:
        f.write('model_checkpoint_path: "%s"\n' % latest)
        for a in allp:
            f.write('all_model_checkpoint_paths: "%s"\n' % a)
    os.replace(tmp, os.path.join(save_dir, INDEX))


def save_checkpoint(save_dir: str, step: int, model: torch.nn.Module, optimizer=None, cfg=None,
                    extra: Optional[Dict[str, Any]] = None, state: Optional[Dict[str, torch.Tensor]] = None,
                    keep: int = 5) -> str:
    os.makedirs(save_dir, exist_ok=True)
    name = "model.ckpt-%d" % step
    tensors = {"model/" + k: v.detach().to("cpu", torch.float32).contiguous().clone()
               for k, v in model.state_dict().items()}
    if optimizer is not None:
        for k, v in optimizer.state_dict().items():
            if torch.is_tensor(v):
                tensors["optim/" + k] = v.detach().cpu().contiguous().clone()
    for k, v in (state or {}).items():
        tensors["state/" + k] = v.detach().cpu().contiguous().clone()
    meta = {"format": "skrnn-ckpt-v1", "step": str(step),
            "extra": json.dumps(extra or {}),
            "optim_step_count": str(getattr(optimizer, "step_count", 0))}
    if cfg is not None:
        meta["config"] = json.dumps(cfg.to_dict())
        from ..config import save_json
        save_json(cfg, os.path.join(save_dir, "config.json"))
    path = os.path.join(save_dir, name + ".safetensors")
    tmp = path + ".tmp"
    save_file(tensors, tmp, metadata=meta)
    os.replace(tmp, path)
    _, allp = _read_index(save_dir)
    allp = [a for a in allp if a != name] + [name]
    for old in allp[:-keep] if keep > 0 else []:
        try:
            os.remove(os.path.join(save_dir, old + ".safetensors"))
        except FileNotFoundError:
            pass
    allp = allp[-keep:] if keep > 0 else allp
    _write_index(save_dir, name, allp)
    return path


def latest_checkpoint(save_dir: str) -> Optional[str]:
    latest, _ = _read_index(save_dir)
    if latest is None:
        return None
    p = os.path.join(save_dir, latest + ".safetensors")
    return p if os.path.exists(p) else None


def read_metadata(path: str) -> Dict[str, str]:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        return dict(f.metadata() or {})


def load_checkpoint(path: str, model: torch.nn.Module, optimizer=None, strict: bool = True):
    """Load weights (and optimizer state) in place. Returns
    ``(step, extra, state_tensors)``."""
    t = load_file(path, device="cpu")
    meta = read_metadata(path)
    sd = {k[len("model/"):]: v for k, v in t.items() if k.startswith("model/")}
    with torch.no_grad():
        own = model.state_dict()
        missing = [k for k in own if k not in sd]
        if strict and missing:
            raise KeyError("checkpoint is missing %s" % missing)
        for k, v in own.items():
            if k in sd:
                v.copy_(sd[k].to(v.dtype))
    from ..ops import gemm
    gemm.invalidate_derived()
    if optimizer is not None and "optim/m" in t:
        osd = {k[len("optim/"):]: v.to(optimizer.m.device) for k, v in t.items() if k.startswith("optim/")}
        osd["step_count"] = int(meta.get("optim_step_count", "0"))
        optimizer.load_state_dict(osd)
    state = {k[len("state/"):]: v for k, v in t.items() if k.startswith("state/")}
    return int(meta.get("step", "0")), json.loads(meta.get("extra", "{}")), state


def load_config(save_dir: str):
    from ..config import load_json
    return load_json(os.path.join(save_dir, "config.json"))
