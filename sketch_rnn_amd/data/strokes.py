"""Stroke formats and conversions.

Two stroke-5 layouts exist in this framework:

* **reference** layout (``model.py:43,104``, ``utils.py:232``):
  ``[dx, dy, eos, eoc, cont]`` -- eos = end of stroke (pen lifts after the
  point), eoc = end of character, cont = pen stays down;
* **magenta** layout (sketch-rnn VAE): ``[dx, dy, p1, p2, p3]`` -- p1 = pen
  down (continue), p2 = pen up after this point, p3 = end of sketch.

They carry the same information up to a permutation of the one-hot columns:
reference ``(eos, eoc, cont)`` == magenta ``(p2, p3, p1)``.

Stroke-3 is ``[dx, dy, pen_lift]`` (QuickDraw ``.npz`` format).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np

# column permutations between the two stroke-5 layouts
_REF_FROM_MAG = [0, 1, 3, 4, 2]   # ref[:, k] = mag[:, _REF_FROM_MAG[k]]
_MAG_FROM_REF = [0, 1, 4, 2, 3]   # mag[:, k] = ref[:, _MAG_FROM_REF[k]]

START_TOKEN_MAGENTA = np.array([0, 0, 1, 0, 0], dtype=np.float32)


def reference_to_magenta(s5: np.ndarray) -> np.ndarray:
    """``[dx,dy,eos,eoc,cont]`` -> ``[dx,dy,p1,p2,p3]`` (lossless)."""
    return np.asarray(s5)[..., _MAG_FROM_REF]


def magenta_to_reference(s5: np.ndarray) -> np.ndarray:
    """``[dx,dy,p1,p2,p3]`` -> ``[dx,dy,eos,eoc,cont]`` (lossless)."""
    return np.asarray(s5)[..., _REF_FROM_MAG]


def stroke4_to_stroke3(s4: np.ndarray) -> np.ndarray:
    """Reference cache rows ``[dx,dy,eos,eoc]`` -> stroke-3 ``[dx,dy,lift]``."""
    s4 = np.asarray(s4)
    out = np.zeros((len(s4), 3), dtype=np.float32)
    out[:, 0:2] = s4[:, 0:2]
    out[:, 2] = np.maximum(s4[:, 2], s4[:, 3])
    return out


def to_big_strokes(stroke: np.ndarray, max_len: int = 250) -> np.ndarray:
    """stroke-3 -> magenta stroke-5 padded to ``max_len`` (no start token)."""
    result = np.zeros((max_len, 5), dtype=np.float32)
    n = len(stroke)
    assert n <= max_len
    result[0:n, 0:2] = stroke[:, 0:2]
    result[0:n, 3] = stroke[:, 2]
    result[0:n, 2] = 1 - result[0:n, 3]
    result[n:, 4] = 1
    return result


def to_normal_strokes(big_stroke: np.ndarray) -> np.ndarray:
    """magenta stroke-5 -> stroke-3, cut at the first end-of-sketch."""
    big_stroke = np.asarray(big_stroke)
    hits = np.nonzero(big_stroke[:, 4] > 0)[0]
    n = int(hits[0]) if len(hits) and hits[0] > 0 else len(big_stroke)
    result = np.zeros((n, 3), dtype=np.float32)
    result[:, 0:2] = big_stroke[0:n, 0:2]
    result[:, 2] = big_stroke[0:n, 3]
    return result


def clean_strokes(sample_strokes, factor: float = 100) -> List[List[int]]:
    """Cut after end-of-sketch, scale to pixels, integerize (JSON export)."""
    out = []
    for row in sample_strokes:
        if int(row[4]) != 0:
            break
        out.append([int(round(row[0] * factor)), int(round(row[1] * factor)), int(row[2]), int(row[3]), 0])
    out.append([0, 0, 0, 0, 1])
    return out


def strokes_to_lines(strokes: np.ndarray) -> List[List[List[float]]]:
    """stroke-3 -> list of absolute polylines."""
    x = y = 0.0
    lines, line = [], []
    for dx, dy, lift in np.asarray(strokes, dtype=np.float64):
        x += dx
        y += dy
        line.append([x, y])
        if lift == 1:
            lines.append(line)
            line = []
    return lines


def lines_to_strokes(lines) -> np.ndarray:
    """list of absolute polylines -> stroke-3."""
    rows = [[0.0, 0.0, 0.0]]
    for line in lines:
        for i, (x, y) in enumerate(line):
            rows.append([x, y, 1.0 if i == len(line) - 1 else 0.0])
    arr = np.array(rows, dtype=np.float64)
    arr[1:, 0:2] -= arr[:-1, 0:2].copy()
    return arr[1:]


def get_bounds(data: np.ndarray, factor: float = 10) -> Tuple[float, float, float, float]:
    """(min_x, max_x, min_y, max_y) of the cumulative path of stroke-3 data."""
    xy = np.cumsum(np.asarray(data, dtype=np.float64)[:, 0:2] / factor, axis=0)
    xy = np.vstack([np.zeros((1, 2)), xy])
    return float(xy[:, 0].min()), float(xy[:, 0].max()), float(xy[:, 1].min()), float(xy[:, 1].max())


def augment_strokes(strokes: np.ndarray, prob: float, rng: np.random.RandomState) -> np.ndarray:
    """Randomly merge interior points of a stroke (never stroke ends)."""
    result = []
    prev = [0.0, 0.0, 1.0]
    count = 0
    stroke = [0.0, 0.0, 1.0]
    for row in strokes:
        cand = [float(row[0]), float(row[1]), float(row[2])]
        if cand[2] == 1 or prev[2] == 1:
            count = 0
        else:
            count += 1
        u = rng.rand()
        if cand[2] == 0 and prev[2] == 0 and count > 2 and u < prob:
            stroke[0] += cand[0]
            stroke[1] += cand[1]
        else:
            stroke = cand
            prev = stroke
            result.append(stroke)
    return np.array(result, dtype=np.float32)


def random_scale(data: np.ndarray, factor: float, rng: np.random.RandomState) -> np.ndarray:
    sx = (rng.random_sample() - 0.5) * 2 * factor + 1.0
    sy = (rng.random_sample() - 0.5) * 2 * factor + 1.0
    out = np.array(data, dtype=np.float32, copy=True)
    out[:, 0] *= sx
    out[:, 1] *= sy
    return out


def pad_batch_magenta(batch: Sequence[np.ndarray], max_len: int) -> np.ndarray:
    """stroke-3 list -> ``[B, max_len + 1, 5]`` magenta stroke-5 with S0 token."""
    out = np.zeros((len(batch), max_len + 1, 5), dtype=np.float32)
    for i, s in enumerate(batch):
        n = len(s)
        assert n <= max_len
        out[i, 1:n + 1, 0:2] = s[:, 0:2]
        out[i, 1:n + 1, 3] = s[:, 2]
        out[i, 1:n + 1, 2] = 1 - s[:, 2]
        out[i, n + 1:, 4] = 1
        out[i, 0] = START_TOKEN_MAGENTA
    return out
