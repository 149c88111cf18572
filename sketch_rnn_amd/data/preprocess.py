"""SVG corpus -> stroke-4 cache (reference capability R4, ``utils.py:124-217``).

Walks a directory tree, reads every ``*.svg`` file, collects the ``d``
attribute of every element, flattens line and cubic-Bezier segments into
points and delta-encodes them into ``[dx, dy, eos, eoc]`` rows (float32).

Behaviour pinned to the reference:

* only ``Line`` and ``CubicBezier`` segments are used, other kinds are
  reported and skipped (``utils.py:160-163``);
* a cubic is sampled at ``n + 1`` Bernstein points with
  ``n = clamp(int(chord / 10) + 1, 1, 3)`` (``utils.py:173-178``);
* the start point is emitted only for segment index 0 of each path, the
  ``eos`` flag only on the final point of the final segment of a path
  (``utils.py:181-189``);
* rows are delta-encoded in float32, the last row gets ``eoc = 1`` and the
  first (absolute) row is dropped (``utils.py:190-195``).

The cache is written as an ``.npz`` of a flat float32 point array plus int64
offsets (no pickle), see :func:`save_stroke_cache`.
"""
from __future__ import annotations

import os
import sys
import xml.etree.ElementTree as ET
from typing import List, Sequence, Tuple

import numpy as np

from .svgpath import CubicBezier, Line, parse_path


def cubic_bezier_points(x0, y0, x1, y1, x2, y2, x3, y3, n: int = 20) -> List[Tuple[float, float]]:
    """``n + 1`` evenly spaced (in t) points on a cubic Bezier."""
    pts = []
    for i in range(n + 1):
        t = float(i) / float(n)
        u = 1.0 - t
        a, b, c, d = u ** 3, 3.0 * t * u ** 2, 3.0 * t ** 2 * u, t ** 3
        pts.append((a * x0 + b * x1 + c * x2 + d * x3, a * y0 + b * y1 + c * y2 + d * y3))
    return pts


def svg_path_strings(svgfile: str) -> List[str]:
    tree = ET.parse(svgfile)
    return [el.attrib["d"] for el in tree.iter() if "d" in el.attrib]


def build_lines(svgfile: str, line_length_threshold: float = 10.0, min_points_per_path: int = 1,
                max_points_per_path: int = 3, length_log: list | None = None,
                verbose: bool = False) -> np.ndarray:
    """Convert one SVG file into a ``[N, 4]`` float32 stroke array."""
    rows: List[List[float]] = []
    for d in svg_path_strings(svgfile):
        path = parse_path(d)
        nseg = len(path)
        for i, seg in enumerate(path):
            if type(seg) not in (Line, CubicBezier):
                if verbose:
                    print("skipping non line/cubic segment: %r" % (seg,), file=sys.stderr)
                continue
            xs, ys, xe, ye = seg.start.real, seg.start.imag, seg.end.real, seg.end.imag
            chord = float(np.sqrt((xe - xs) * (xe - xs) + (ye - ys) * (ye - ys)))
            if length_log is not None:
                length_log.append(chord)
            if type(seg) is CubicBezier:
                n = int(chord / line_length_threshold) + 1
                n = min(max(n, min_points_per_path), max_points_per_path)
                pts = cubic_bezier_points(xs, ys, seg.control1.real, seg.control1.imag,
                                          seg.control2.real, seg.control2.imag, xe, ye, n)
            else:
                pts = [(xs, ys), (xe, ye)]
            if i == 0:
                rows.append([pts[0][0], pts[0][1], 0.0, 0.0])
            last = len(pts) - 1
            for j in range(1, len(pts)):
                eos = 1.0 if (j == last and i == nseg - 1) else 0.0
                rows.append([pts[j][0], pts[j][1], eos, 0.0])
    if len(rows) < 2:
        return np.zeros((0, 4), dtype=np.float32)
    lines = np.array(rows, dtype=np.float32)
    lines[1:, 0:2] -= lines[0:-1, 0:2]
    lines[-1, 3] = 1.0
    lines[0] = 0.0
    return lines[1:]


def list_svg_files(data_dir: str) -> List[str]:
    files = []
    for dirname, _subdirs, fnames in os.walk(data_dir):
        for fname in fnames:
            files.append(dirname + "/" + fname)
    return [f for f in files if f[-3:] == "svg"]


def preprocess(data_dir: str, out_file: str | None = None, verbose: bool = False):
    """Build stroke arrays for every SVG under ``data_dir``.

    Returns ``(sketches, length_data)``; writes the cache when ``out_file``.
    """
    length_data: list = []
    sketches = []
    for f in list_svg_files(data_dir):
        if verbose:
            print("processing " + f)
        arr = build_lines(f, length_log=length_data, verbose=verbose)
        if len(arr):
            sketches.append(arr)
    if out_file is not None:
        save_stroke_cache(out_file, sketches)
    return sketches, length_data


def save_stroke_cache(path: str, sketches: Sequence[np.ndarray]) -> None:
    """Pickle-free cache: flat ``points[total, C]`` + ``offsets[n + 1]``."""
    offsets = np.zeros(len(sketches) + 1, dtype=np.int64)
    for k, s in enumerate(sketches):
        offsets[k + 1] = offsets[k] + len(s)
    width = sketches[0].shape[1] if len(sketches) else 4
    pts = np.concatenate(sketches, axis=0).astype(np.float32) if len(sketches) else np.zeros((0, width), np.float32)
    tmp = path + ".tmp.npz"
    np.savez(tmp, points=pts, offsets=offsets)
    os.replace(tmp, path)


def load_stroke_cache(path: str) -> List[np.ndarray]:
    with np.load(path, allow_pickle=False) as z:
        pts, off = z["points"], z["offsets"]
    return [pts[off[k]:off[k + 1]].copy() for k in range(len(off) - 1)]
