"""Data pipeline: SVG preprocessing (R4), cache (R5), reference packer (R6)
quirks pinned as golden tests, native-vs-oracle packer
parity, DP sharding, stroke-format converters, the Magenta-style dataset and
the synthetic generator."""
import os
import sys

import numpy as np
import pytest

from sketch_rnn_amd.data import strokes as S
from sketch_rnn_amd.data.dataset import StrokeDataset
from sketch_rnn_amd.data.loader import SketchLoader, _Cursor, pack_rows_reference
from sketch_rnn_amd.data.preprocess import build_lines, load_stroke_cache, preprocess, save_stroke_cache
from sketch_rnn_amd.data.synthetic import synthetic_corpus, synthetic_reference_corpus
from sketch_rnn_amd.utils import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="session")
def host_lib():
    if native.host_lib() is None:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import build_native
        build_native.build_host()
    lib = native.host_lib()
    assert lib is not None
    return lib


SVG = """<svg xmlns="http://www.w3.org/2000/svg">
<g><path d="M0,0 L30,0 L30,40"/></g>
<path d="M-10,-10 C-10,20 20,20 20,-10"/>
<path d="M0,0 Q10,10 20,0"/>
</svg>"""


def test_build_lines_golden(tmp_path):
    # SURVEY.md §3.4 [verified]: 3-vertex line path, cubic with chord 30
    # (-> 3 segments), quadratic skipped; path start dropped; pen-up move
    # carries eos=0; last row eos=eoc=1.
    f = tmp_path / "a.svg"
    f.write_text(SVG)
    rows = build_lines(str(f))
    exp = np.array([[30, 0, 0, 0], [0, 40, 1, 0], [-40, -50, 0, 0], [7.7777777, 20, 0, 0],
                    [14.444444, 0, 0, 0], [7.7777777, -20, 1, 1]], np.float32)
    assert rows.dtype == np.float32
    np.testing.assert_allclose(rows, exp, atol=1e-4)


def test_preprocess_walk_and_cache(tmp_path):
    d = tmp_path / "kanji"
    (d / "sub").mkdir(parents=True)
    (d / "a.svg").write_text(SVG)
    (d / "sub" / "b.svg").write_text(SVG.replace("L30,40", "L30,40 L0,40"))
    (d / "notes.txt").write_text("ignored")
    out = tmp_path / "kanji.npz"
    sk, lengths = preprocess(str(d), str(out))
    assert len(sk) == 2 and sorted(len(s) for s in sk) == [6, 7]
    # chord lengths of every line/cubic segment (quadratic skipped, not logged)
    assert sorted(lengths)[:2] == [30.0, 30.0] and len(lengths) == 3 + 4
    back = load_stroke_cache(str(out))
    for a, b in zip(sk, back):
        np.testing.assert_array_equal(a, b)


def test_cache_roundtrip_no_pickle(tmp_path):
    sk = [np.random.RandomState(i).randn(5 + i, 4).astype(np.float32) for i in range(4)]
    p = str(tmp_path / "c.npz")
    save_stroke_cache(p, sk)
    with np.load(p, allow_pickle=False) as z:
        assert set(z.files) == {"points", "offsets"} and z["points"].dtype == np.float32
    for a, b in zip(sk, load_stroke_cache(p)):
        np.testing.assert_array_equal(a, b)


def _sk(n, start=0.0):
    a = np.zeros((n, 4), np.float32)
    a[:, 0] = np.arange(n) + start
    a[:, 1] = -np.arange(n)
    a[n // 2, 2] = 1.0
    a[-1, 2:4] = 1.0
    return a


def test_packer_off_by_one_golden():
    # SURVEY.md §5.9 [verified]: sketches of lengths 4 and 3 emit 3 and 2 points;
    # the last emitted point of each is relabelled eoc (eos=cont=0).
    sk = [_sk(4, 0.0), _sk(3, 100.0)]
    cur = _Cursor(2)
    out = pack_rows_reference(sk, np.array([0, 1]), cur, 1, 6, np.ones((1, 2)))
    row = out[0]
    np.testing.assert_array_equal(row[:, 0], [0, 1, 2, 100, 101, 0])
    np.testing.assert_array_equal(row[:, 2:5], [[0, 0, 1], [0, 0, 1], [0, 1, 0], [0, 0, 1], [0, 1, 0], [0, 0, 1]])
    # 2 sketches consumed -> wrapped; one more tick after the row
    assert cur.epoch_finished and cur.pointer == 1


def test_packer_row_starts_and_scale():
    sk = [_sk(5, 10.0 * k) for k in range(7)]
    cur = _Cursor(7)
    sc = np.array([[0.5, 2.0], [1.0, 1.0], [1.0, 3.0]])
    out = pack_rows_reference(sk, np.arange(7), cur, 3, 5, sc)
    # row 0 packs sketch0 (4 pts) + first pt of sketch1; pointer ticks to 2 at row end
    np.testing.assert_allclose(out[0, :, 0], np.array([0, 1, 2, 3, 10]) * 0.5)
    np.testing.assert_allclose(out[0, :, 1], np.array([0, -1, -2, -3, 0]) * 2.0)
    assert out[1, 0, 0] == 20.0  # row 1 starts at the start of sketch 2
    assert out[2, 0, 0] == 40.0
    assert np.all(out[:, :, 2:5].sum(-1) == 1)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_native_packer_matches_oracle(host_lib, seed):
    sk = synthetic_reference_corpus(37, seed=seed, max_len=60)
    a = SketchLoader(8, 50, scale_factor=15.0, sketches=sk, seed=seed, use_native=True)
    b = SketchLoader(8, 50, scale_factor=15.0, sketches=sk, seed=seed, use_native=False)
    assert a._native is not None and b._native is None
    for _ in range(25):  # crosses several epoch boundaries
        xa, ya = a.next_batch()
        xb, yb = b.next_batch()
        np.testing.assert_array_equal(xa, xb)
        np.testing.assert_array_equal(ya, yb)
        assert a.pointer == b.pointer and a.epoch_finished == b.epoch_finished
        if a.epoch_finished:
            a.reset_index_pointer()
            b.reset_index_pointer()


def test_loader_teacher_forcing_and_scaling():
    sk = synthetic_reference_corpus(10, seed=3, max_len=40)
    ld = SketchLoader(4, 20, scale_factor=15.0, sketches=sk, seed=0, use_native=False)
    np.testing.assert_allclose(ld.raw_data[0][:, :2], sk[0][:, :2] / 15.0, rtol=1e-6)
    full = ld.next_batch_full()
    ld2 = SketchLoader(4, 20, scale_factor=15.0, sketches=sk, seed=0, use_native=False)
    x, y = ld2.next_batch()
    np.testing.assert_array_equal(x, full[:, :-1])
    np.testing.assert_array_equal(y, full[:, 1:])
    assert x.shape == (4, 20, 5)


def test_loader_dp_sharding_disjoint():
    sk = synthetic_reference_corpus(23, seed=1, max_len=30)
    lds = [SketchLoader(2, 10, sketches=sk, seed=7, rank=r, world_size=3, use_native=False) for r in range(3)]
    perms = [set(ld._perm.tolist()) for ld in lds]
    assert set().union(*perms) == set(range(23))
    assert sum(len(p) for p in perms) == 23
    assert not (perms[0] & perms[1]) and not (perms[1] & perms[2])


def test_epoch_reset_reshuffles_previous_permutation():
    sk = synthetic_reference_corpus(12, seed=1, max_len=30)
    ld = SketchLoader(2, 10, sketches=sk, seed=11, use_native=False)
    rng = np.random.RandomState(11)
    p1 = rng.permutation(np.arange(12))
    np.testing.assert_array_equal(ld.index, p1)
    ld.reset_index_pointer()
    np.testing.assert_array_equal(ld.index, rng.permutation(p1))


def test_format_converters_roundtrip():
    rng = np.random.RandomState(0)
    s5 = np.zeros((9, 5), np.float32)
    s5[:, :2] = rng.randn(9, 2)
    s5[:, 4] = 1
    s5[3, 4], s5[3, 2] = 0, 1
    s5[8, 4], s5[8, 3] = 0, 1
    m = S.reference_to_magenta(s5)
    np.testing.assert_array_equal(S.magenta_to_reference(m), s5)
    # reference [eos, eoc, cont] -> magenta [p1=down, p2=up, p3=end]
    assert m[0, 2] == 1 and m[3, 3] == 1 and m[8, 4] == 1


def test_big_normal_strokes_and_lines():
    s3 = np.array([[1, 2, 0], [3, 4, 1], [-1, 0, 0], [2, 2, 1]], np.float32)
    big = S.to_big_strokes(s3, max_len=8)
    assert big.shape == (8, 5)
    assert big[4:, 4].sum() == 4 and big[:4, 4].sum() == 0
    np.testing.assert_allclose(S.to_normal_strokes(big), s3)
    lines = S.strokes_to_lines(s3)
    assert len(lines) == 2
    np.testing.assert_allclose(S.lines_to_strokes(lines), s3)  # absolute from the origin: exact inverse


def test_pad_batch_magenta():
    s3 = [np.array([[1, 1, 0], [2, 2, 1]], np.float32), np.array([[1, 0, 1]], np.float32)]
    out = S.pad_batch_magenta(s3, 4)
    assert out.shape == (2, 5, 5)
    np.testing.assert_array_equal(out[:, 0], [[0, 0, 1, 0, 0]] * 2)  # S0 token
    np.testing.assert_array_equal(out[0, 1:3, :2], [[1, 1], [2, 2]])
    np.testing.assert_array_equal(out[0, 1:3, 2:], [[1, 0, 0], [0, 1, 0]])
    np.testing.assert_array_equal(out[0, 3:, 2:], [[0, 0, 1]] * 2)
    np.testing.assert_array_equal(out[1, 2:, 2:], [[0, 0, 1]] * 3)


def test_augment_and_scale_deterministic():
    s3 = np.abs(np.random.RandomState(0).randn(40, 3)).astype(np.float32)
    s3[:, 2] = (np.arange(40) % 7 == 6)
    a = S.augment_strokes(s3, 0.3, np.random.RandomState(5))
    b = S.augment_strokes(s3, 0.3, np.random.RandomState(5))
    np.testing.assert_array_equal(a, b)
    assert len(a) <= len(s3)
    np.testing.assert_allclose(a[:, :2].sum(0), s3[:, :2].sum(0), rtol=1e-4)  # dropping merges offsets
    r = S.random_scale(s3, 0.15, np.random.RandomState(1))
    assert r.shape == s3.shape and not np.allclose(r, s3)


def test_stroke_dataset_batches_and_normalize():
    s, l = synthetic_corpus(64, seed=0, max_len=50, n_classes=3)
    ds = StrokeDataset(s, 16, 50, labels=l, seed=0)
    scale = ds.normalize()
    assert scale > 0
    flat = np.concatenate([x[:, :2].ravel() for x in ds.strokes])
    assert abs(np.std(flat) - 1.0) < 0.05
    x, lens, lab = ds.get_batch(0)
    assert x.shape == (16, 51, 5) and lens.shape == (16,) and lab.shape == (16,)
    assert np.all(lens <= 50) and np.all(lens >= 1)
    for b in range(16):
        assert np.all(x[b, lens[b] + 1:, 4] == 1)
    # DP (weak scaling): rank r takes slice r of one global batch of 16*world
    dss = []
    for _ in range(3):
        d = StrokeDataset(s, 16, 50, labels=l, seed=0)
        d.normalize()
        dss.append(d)
    xa = dss[0].random_batch(0, 2)[0]
    xb = dss[1].random_batch(1, 2)[0]
    xg = dss[2].random_batch(0, 1, batch_size=32)[0]
    assert xa.shape[0] == 16 and xb.shape[0] == 16
    np.testing.assert_array_equal(np.concatenate([xa, xb]), xg)


def test_synthetic_corpus_shape_and_determinism():
    a, la = synthetic_corpus(20, seed=4, max_len=100, n_classes=5)
    b, lb = synthetic_corpus(20, seed=4, max_len=100, n_classes=5)
    assert len(a) == 20 and all(x.shape[1] == 3 for x in a)
    assert all(len(x) <= 100 for x in a) and set(np.asarray(la).tolist()) <= set(range(5))
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert all(x[-1, 2] == 1 for x in a)
