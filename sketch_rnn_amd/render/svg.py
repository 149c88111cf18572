"""SVG rendering of stroke sequences (reference capability R18, ``utils.py:10-103``).

No third-party SVG library: documents are assembled as text.

* :func:`calculate_start_point` -- cumulative (rounded to 3 dp) offsets,
  bounding box from the origin and the offset that centres the sketch in a
  ``block_size`` cell (``utils.py:10-30``).
* :func:`draw_stroke_color_array` -- a grid of ``maxcol`` columns, white
  background, one ``<path>`` per segment, pen lifted after ``eos`` or
  ``eoc``, a random RGB colour in ``[0, 225]`` per stroke (black when
  ``color_mode`` is off) (``utils.py:32-83``).
* :func:`draw_stroke_color` -- splits a long stream at each ``eoc`` (the
  trailing stub without ``eoc`` is dropped) and renders the pieces as a grid
  (``utils.py:85-103``).
* :func:`draw_strokes3` / :func:`grid_strokes3` -- the same for stroke-3
  sketches (VAE samples), one ``<path>`` per pen-down polyline.

Inputs use the reference layout ``[dx, dy, eos, eoc, cont]`` unless noted.
"""
from __future__ import annotations

import math
import random as _random
from typing import List, Optional, Sequence, Tuple

import numpy as np

MAX_COLOR = 225


def calculate_start_point(data, factor: float = 1.0, block_size: float = 200) -> Tuple[float, float, float, float]:
    sx = sy = 0.0
    maxx = minx = maxy = miny = 0.0
    for row in np.asarray(data):
        sx += round(float(row[0]) * factor, 3)
        sy += round(float(row[1]) * factor, 3)
        maxx, minx = max(maxx, sx), min(minx, sx)
        maxy, miny = max(maxy, sy), min(miny, sy)
    abs_x = block_size / 2 - (maxx - minx) / 2 - minx
    abs_y = block_size / 2 - (maxy - miny) / 2 - miny
    return abs_x, abs_y, (maxx - minx), (maxy - miny)


def _num(v: float) -> str:
    return repr(float(v)) if not float(v).is_integer() else str(float(v))


class SvgDoc:
    def __init__(self, width: float, height: float):
        self.width, self.height = width, height
        self.items: List[str] = []

    def rect(self, x, y, w, h, fill="white"):
        self.items.append('<rect fill="%s" height="%s" width="%s" x="%s" y="%s" />' % (fill, _num(h), _num(w), _num(x), _num(y)))

    def path(self, d: str, stroke: str, width: float, fill: Optional[str] = None):
        self.items.append('<path d="%s" fill="%s" stroke="%s" stroke-width="%s" />' % (
            d.strip(), fill if fill is not None else stroke, stroke, _num(width)))

    def tostring(self) -> str:
        head = ('<?xml version="1.0" encoding="utf-8" ?>\n<svg baseProfile="full" height="%s" version="1.1" '
                'width="%s" xmlns="http://www.w3.org/2000/svg" xmlns:ev="http://www.w3.org/2001/xml-events" '
                'xmlns:xlink="http://www.w3.org/1999/xlink"><defs />' % (_num(self.height), _num(self.width)))
        return head + "".join(self.items) + "</svg>"

    def save(self, filename: str):
        with open(filename, "w") as f:
            f.write(self.tostring())


def _rand_color(rng) -> str:
    return "rgb(%d,%d,%d)" % (rng.randint(0, MAX_COLOR), rng.randint(0, MAX_COLOR), rng.randint(0, MAX_COLOR))


def draw_stroke_color_array(data: Sequence, factor: float = 1, svg_filename: Optional[str] = "sample.svg",
                            stroke_width: float = 1, block_size: float = 200, maxcol: int = 5,
                            color_mode: bool = True, rng: Optional[_random.Random] = None) -> Optional[SvgDoc]:
    num_char = len(data)
    if num_char < 1:  # nothing accepted: still emit a (blank) canvas
        doc = SvgDoc(block_size, block_size)
        doc.rect(0, 0, block_size, block_size, "white")
        if svg_filename:
            doc.save(svg_filename)
        return doc
    rng = rng or _random.Random()
    numrow = math.ceil(num_char / maxcol)
    w, h = block_size * min(num_char, maxcol), block_size * numrow
    doc = SvgDoc(w, h)
    doc.rect(0, 0, w, h, "white")
    color = _rand_color(rng)
    for j, cdata in enumerate(data):
        cdata = np.asarray(cdata)
        lift_pen = 0.0
        abs_x, abs_y, _, _ = calculate_start_point(cdata, factor, block_size)
        abs_x += (j % maxcol) * block_size
        abs_y += (j // maxcol) * block_size
        for row in cdata:
            x = round(float(row[0]) * factor, 3)
            y = round(float(row[1]) * factor, 3)
            prev_x, prev_y = round(abs_x, 3), round(abs_y, 3)
            abs_x += x
            abs_y += y
            if lift_pen == 1:
                d = "M %s,%s " % (abs_x, abs_y)
                color = _rand_color(rng)
            else:
                d = "M %s,%s L %s,%s " % (prev_x, prev_y, abs_x, abs_y)
            lift_pen = max(float(row[2]), float(row[3]))
            doc.path(d, color if color_mode else "#000", stroke_width)
    if svg_filename:
        doc.save(svg_filename)
    return doc


def split_sketch(data) -> List[np.ndarray]:
    """Split a stream at each eoc (inclusive); the trailing stub is dropped."""
    data = np.asarray(data, dtype=np.float32)
    out, start = [], 0
    for i in range(len(data)):
        if data[i, 3] > 0:
            out.append(data[start:i + 1])
            start = i + 1
    return out


def draw_stroke_color(data, factor=1, svg_filename="sample.svg", stroke_width=1, block_size=200, maxcol=5,
                      color_mode=True, rng=None):
    return draw_stroke_color_array(split_sketch(data), factor, svg_filename, stroke_width, block_size, maxcol,
                                   color_mode, rng)


# ----------------------------------------------------------------------------
# stroke-3 (VAE) rendering
# ----------------------------------------------------------------------------
def _bounds3(s3: np.ndarray, factor: float):
    xy = np.cumsum(np.asarray(s3, dtype=np.float64)[:, 0:2] / factor, axis=0)
    xy = np.vstack([np.zeros((1, 2)), xy])
    return xy[:, 0].min(), xy[:, 0].max(), xy[:, 1].min(), xy[:, 1].max()


def _polyline_paths(s3: np.ndarray, factor: float, ox: float, oy: float) -> List[str]:
    paths, cur = [], ["M %.3f,%.3f" % (ox, oy)]
    x, y = ox, oy
    lift = 1.0
    for dx, dy, pen in np.asarray(s3, dtype=np.float64):
        x += dx / factor
        y += dy / factor
        cur.append(("M" if lift == 1 else "L") + " %.3f,%.3f" % (x, y))
        lift = pen
        if pen == 1:
            paths.append(" ".join(cur))
            cur = []
    if len(cur) > 1:
        paths.append(" ".join(cur))
    return paths


def grid_strokes3(sketches: Sequence[np.ndarray], svg_filename: Optional[str] = "grid.svg", factor: float = 0.2,
                  block_size: float = 160, maxcol: int = 5, stroke_width: float = 1.0, color: str = "black"):
    """Grid of stroke-3 sketches, each centred in its cell."""
    n = len(sketches)
    if n == 0:
        return None
    rows = math.ceil(n / maxcol)
    doc = SvgDoc(block_size * min(n, maxcol), block_size * rows)
    doc.rect(0, 0, doc.width, doc.height, "white")
    for k, s3 in enumerate(sketches):
        minx, maxx, miny, maxy = _bounds3(s3, factor)
        ox = (k % maxcol) * block_size + block_size / 2 - (maxx + minx) / 2
        oy = (k // maxcol) * block_size + block_size / 2 - (maxy + miny) / 2
        for d in _polyline_paths(s3, factor, ox, oy):
            doc.path(d, color, stroke_width, fill="none")
    if svg_filename:
        doc.save(svg_filename)
    return doc


def draw_strokes3(s3: np.ndarray, svg_filename: Optional[str] = "sample.svg", factor: float = 0.2,
                  stroke_width: float = 1.0):
    minx, maxx, miny, maxy = _bounds3(s3, factor)
    w, h = 50 + maxx - minx, 50 + maxy - miny
    doc = SvgDoc(w, h)
    doc.rect(0, 0, w, h, "white")
    for d in _polyline_paths(s3, factor, 25 - minx, 25 - miny):
        doc.path(d, "black", stroke_width, fill="none")
    if svg_filename:
        doc.save(svg_filename)
    return doc
