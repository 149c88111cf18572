"""SVG renderer (R18) against the reference's own showcase artefact
``example/output.svg`` (20 samples, 5 x 4 grid of 160 px cells, 1365 paths):
the strokes are recovered from that file's path coordinates, re-rendered with
our renderer, and every segment must land on the same coordinates (same
centring, same 3-dp rounding, same pen-lift rule)."""
import os
import re

import numpy as np
import pytest

from sketch_rnn_amd.render.svg import (calculate_start_point, draw_stroke_color, draw_stroke_color_array,
                                       grid_strokes3, split_sketch)

REF_SVG = "/root/reference/example/output.svg"
_PATH = re.compile(r'<path d="([^"]*)"')


def _parse(svg: str):
    segs = []
    for d in _PATH.findall(svg):
        nums = [float(v) for v in re.findall(r"-?\d+(?:\.\d+)?(?:e-?\d+)?", d)]
        segs.append(nums)
    return segs


def _recover(segs, block=160.0, maxcol=5):
    """Sketches [dx, dy, eos, eoc, cont] from the reference renderer's output."""
    sketches, cur, start, last_end = [], [], None, None
    for s in segs:
        if len(s) == 4:
            prev, end = (s[0], s[1]), (s[2], s[3])
            # the file holds 12-significant-digit str() values (Python 2), so
            # continuity is checked to within the 3-dp rounding only
            if last_end is None or abs(prev[0] - last_end[0]) > 2e-3 or abs(prev[1] - last_end[1]) > 2e-3:
                if cur:
                    sketches.append((start, cur))
                cur, start, last_end = [], prev, prev
            cur.append([end[0] - last_end[0], end[1] - last_end[1], 0, 0, 1])
            last_end = end
        else:  # pen was lifted after the previous row: move only
            cur[-1][2:] = [1, 0, 0]
            end = (s[0], s[1])
            cur.append([end[0] - last_end[0], end[1] - last_end[1], 0, 0, 1])
            last_end = end
    sketches.append((start, cur))
    return sketches


@pytest.mark.skipif(not os.path.exists(REF_SVG), reason="reference tree not present")
def test_rerender_reference_output_svg(tmp_path):
    svg = open(REF_SVG).read()
    assert 'height="640.0"' in svg and 'width="800"' in svg
    segs = _parse(svg)[0:]
    assert len(segs) == 1365
    sk = _recover(segs)
    assert len(sk) == 20
    data = []
    for j, (start, rows) in enumerate(sk):
        a = np.array(rows, dtype=np.float64)
        a[-1, 2:] = [0, 1, 0]  # sampling stopped at the eoc row
        data.append(a)
        # centring: the recovered start must be what calculate_start_point gives
        ax, ay, _, _ = calculate_start_point(a, 1.0, 160)
        assert abs(ax + (j % 5) * 160 - start[0]) < 2e-3 and abs(ay + (j // 5) * 160 - start[1]) < 2e-3
    doc = draw_stroke_color_array(data, factor=1, svg_filename=str(tmp_path / "o.svg"), stroke_width=2.0,
                                  block_size=160, maxcol=5)
    assert (doc.width, doc.height) == (800, 640)
    ours = _parse(open(tmp_path / "o.svg").read())
    assert len(ours) == len(segs)
    for a, b in zip(ours, segs):
        assert len(a) == len(b)
        assert max(abs(x - y) for x, y in zip(a, b)) < 3e-3, (a, b)


def test_calculate_start_point_and_lift_rule():
    d = np.array([[10, 0, 0, 0, 1], [0, 10, 1, 0, 0], [-20, 0, 0, 0, 1], [0, -20, 0, 1, 0]], np.float32)
    ax, ay, sx, sy = calculate_start_point(d, 1.0, 100)
    assert (sx, sy) == (20.0, 20.0)
    assert (ax, ay) == (100 / 2 - 10 + 10, 100 / 2 - 10 + 10)
    doc = draw_stroke_color_array([d], svg_filename=None, block_size=100, color_mode=False)
    paths = [p for p in doc.items if p.startswith("<path")]
    assert len(paths) == 4
    assert ' L ' not in paths[2] and 'stroke="#000"' in paths[0]  # pen up after the eos row


def test_split_and_grid():
    d = np.zeros((7, 5), np.float32)
    d[:, 4] = 1
    d[2, 3], d[2, 4] = 1, 0
    d[5, 3], d[5, 4] = 1, 0
    parts = split_sketch(d)
    assert [len(p) for p in parts] == [3, 3]  # the stub after the last eoc is dropped
    doc = draw_stroke_color(d, svg_filename=None, block_size=50, maxcol=1)
    assert (doc.width, doc.height) == (50, 100)
    s3 = np.array([[1, 1, 0], [2, 0, 1], [0, 3, 0], [1, 1, 1]], np.float32)
    g = grid_strokes3([s3] * 7, None, factor=1.0, block_size=40, maxcol=3)
    assert (g.width, g.height) == (120, 120)
    assert sum(p.startswith("<path") for p in g.items) == 14
