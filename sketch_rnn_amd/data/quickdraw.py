"""QuickDraw-style stroke-3 corpora.

Two on-disk formats are supported:

* **sketch pack** (``.skpack.npz``, this framework's own, pickle-free): per
  split ``{split}_points`` int16/float32 ``[N, 3]``, ``{split}_offsets``
  int64 ``[n + 1]`` and optional ``{split}_labels``;
* the public QuickDraw ``.npz`` whose ``train/valid/test`` entries are object
  arrays. Those need NumPy's pickle path, so reading one requires the
  caller to pass ``allow_pickle=True`` explicitly for a file they trust;
  :func:`convert_to_pack` turns it into a sketch pack once.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

SPLITS = ("train", "valid", "test")


def save_pack(path: str, splits: Dict[str, Tuple[Sequence[np.ndarray], Sequence[int]]]) -> None:
    arrays = {}
    for name, (strokes, labels) in splits.items():
        off = np.zeros(len(strokes) + 1, dtype=np.int64)
        for k, s in enumerate(strokes):
            off[k + 1] = off[k] + len(s)
        pts = np.concatenate([np.asarray(s, np.float32) for s in strokes], 0) if len(strokes) else \
            np.zeros((0, 3), np.float32)
        arrays[name + "_points"] = pts
        arrays[name + "_offsets"] = off
        arrays[name + "_labels"] = np.asarray(labels, dtype=np.int64)
    np.savez(path, **arrays)


def load_pack(path: str) -> Dict[str, Tuple[List[np.ndarray], np.ndarray]]:
    out = {}
    with np.load(path, allow_pickle=False) as z:
        for name in SPLITS:
            if name + "_points" not in z:
                continue
            pts, off = z[name + "_points"], z[name + "_offsets"]
            labels = z[name + "_labels"] if name + "_labels" in z else np.zeros(len(off) - 1, np.int64)
            out[name] = ([np.asarray(pts[off[k]:off[k + 1]], np.float32) for k in range(len(off) - 1)], labels)
    return out


def load_quickdraw_npz(path: str, allow_pickle: bool = False, label: int = 0):
    """Read a public QuickDraw ``.npz`` (object arrays of stroke-3)."""
    with np.load(path, encoding="latin1", allow_pickle=allow_pickle) as z:
        out = {}
        for name in SPLITS:
            if name in z:
                arr = z[name]
                strokes = [np.asarray(s, dtype=np.float32) for s in arr]
                out[name] = (strokes, np.full(len(strokes), label, dtype=np.int64))
    return out


def convert_to_pack(npz_paths: Sequence[str], out_path: str, allow_pickle: bool = False) -> None:
    merged: Dict[str, Tuple[list, list]] = {s: ([], []) for s in SPLITS}
    for cls, p in enumerate(npz_paths):
        d = load_quickdraw_npz(p, allow_pickle=allow_pickle, label=cls)
        for name, (strokes, labels) in d.items():
            merged[name][0].extend(strokes)
            merged[name][1].extend(labels.tolist())
    save_pack(out_path, merged)
