"""Deterministic synthetic stroke-3 corpora (no network in this environment).

Sketches are built from smooth pen strokes (a heading random walk with
per-class curvature / step statistics) joined by pen-up jumps, so that a
class-conditional model has real signal to learn and a length distribution
similar to QuickDraw (tens to a couple of hundred points, long tail up to
``max_len``).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def synthetic_sketch(rng: np.random.RandomState, max_len: int = 250, cls: int = 0,
                     n_classes: int = 1, target_len: int | None = None) -> np.ndarray:
    # class-specific style: curvature and step length
    curv = 0.15 + 0.6 * ((cls * 0.618) % 1.0)
    step = 6.0 + 10.0 * ((cls * 0.381 + 0.2) % 1.0)
    if target_len is None:
        target_len = int(np.clip(rng.gamma(4.0, 16.0), 8, max_len))
    rows: List[Tuple[float, float, float]] = []
    heading = rng.uniform(0, 2 * np.pi)
    while len(rows) < target_len:
        npts = int(np.clip(rng.poisson(10) + 3, 3, target_len - len(rows))) if target_len - len(rows) >= 3 \
            else target_len - len(rows)
        turn = rng.normal(0.0, curv)
        for k in range(npts):
            heading += turn + rng.normal(0.0, 0.15)
            r = abs(rng.normal(step, step * 0.3))
            rows.append((r * np.cos(heading), r * np.sin(heading), 1.0 if k == npts - 1 else 0.0))
        if len(rows) < target_len:  # pen-up jump to the next stroke start
            heading = rng.uniform(0, 2 * np.pi)
    arr = np.asarray(rows[:target_len], dtype=np.float32)
    arr[-1, 2] = 1.0
    arr[:, 0:2] = np.round(arr[:, 0:2])  # QuickDraw offsets are integers
    return arr


def synthetic_corpus(n: int, seed: int = 0, max_len: int = 250, n_classes: int = 1,
                     include_max: bool = True):
    """Return ``(strokes, labels)``; one sketch is forced to length ``max_len``
    when ``include_max`` so that the padded length equals ``max_len``."""
    rng = np.random.RandomState(seed)
    labels = rng.randint(0, n_classes, size=n)
    strokes = [synthetic_sketch(rng, max_len, int(labels[i]), n_classes) for i in range(n)]
    if include_max and n:
        strokes[0] = synthetic_sketch(rng, max_len, int(labels[0]), n_classes, target_len=max_len)
    return strokes, labels


def synthetic_reference_corpus(n: int, seed: int = 0, max_len: int = 120) -> List[np.ndarray]:
    """Reference-layout ``[dx, dy, eos, eoc]`` sketches (like the kanji cache)."""
    strokes, _ = synthetic_corpus(n, seed=seed, max_len=max_len, include_max=False)
    out = []
    for s in strokes:
        r = np.zeros((len(s), 4), dtype=np.float32)
        r[:, 0:2] = s[:, 0:2]
        r[:, 2] = s[:, 2]
        r[-1, 3] = 1.0
        out.append(r)
    return out
