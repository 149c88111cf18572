"""Reference-mode dataset loader and batch packer (capabilities R5, R6).

``SketchLoader`` mirrors the reference's ``utils.py:105-283`` public surface
(``next_batch``, ``reset_index_pointer``, ``epoch_finished``, ``pointer``,
``num_samples``, ``raw_data``) with these design changes:

* the packing loop runs in native C++ (``csrc/host/packer.cpp`` via
  :mod:`sketch_rnn_amd.utils.native`) over a flat point buffer; a NumPy
  implementation (:func:`pack_rows_reference`) is kept as the oracle and as
  the fallback when the host library is not built;
* randomness comes from an explicit ``numpy.random.RandomState`` (the
  reference uses the global, unseeded NumPy state);
* the cache is a pickle-free ``.npz`` (see :mod:`.preprocess`);
* DP sharding: rank ``r`` of ``W`` walks every W-th entry of the epoch
  permutation so that ranks see disjoint sketches.

Packer semantics reproduced exactly: each row starts at the
beginning of the current sketch, packs consecutive sketches, the point at
``idx == len - 2`` is relabelled ``eoc`` (so the final raw point of a sketch
is never emitted), the pointer ticks once more after each row, and a random
anisotropic scale ``U(0.7, 1.3)`` is applied per row.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence

import numpy as np

from .preprocess import load_stroke_cache, preprocess


class _Cursor:
    """Epoch cursor over a permutation: ``pointer`` / ``epoch_finished``."""

    def __init__(self, n: int):
        self.n = n
        self.pointer = 0
        self.epoch_finished = False

    def tick(self):
        self.pointer += 1
        if self.pointer >= self.n:
            self.pointer = 0
            self.epoch_finished = True


def pack_rows_reference(sketches: Sequence[np.ndarray], index: np.ndarray, cursor: _Cursor,
                        batch_size: int, n: int, scales: np.ndarray) -> np.ndarray:
    """Pure-NumPy packer, semantics of ``utils.py:231-264`` (oracle)."""
    out = np.zeros((batch_size, n, 5), dtype=np.float32)
    for b in range(batch_size):
        res = out[b]
        idx = 0
        data = sketches[index[cursor.pointer]]
        for i in range(n):
            res[i, 0:4] = data[idx]
            res[i, 4] = 1.0
            if res[i, 2] > 0 or res[i, 3] > 0:
                res[i, 4] = 0.0
            idx += 1
            if idx >= len(data) - 1:
                res[i, 4] = 0.0
                res[i, 3] = 1.0
                res[i, 2] = 0.0
                idx = 0
                cursor.tick()
                data = sketches[index[cursor.pointer]]
            assert res[i, 2:5].sum() == 1
        cursor.tick()
        res[:, 0] *= scales[b, 0]
        res[:, 1] *= scales[b, 1]
    return out


class SketchLoader:
    """Packed teacher-forcing batches ``(x[B, T, 5], y[B, T, 5])``.

    Stroke-5 layout is the reference's ``[dx, dy, eos, eoc, cont]``.
    """

    def __init__(self, batch_size: int = 50, seq_length: int = 300, scale_factor: float = 1.0,
                 data_filename: str = "kanji", data_dir: str = "./data",
                 sketches: Optional[List[np.ndarray]] = None, seed: Optional[int] = None,
                 rank: int = 0, world_size: int = 1, use_native: bool = True):
        self.data_dir = data_dir
        self.batch_size = batch_size
        self.seq_length = seq_length
        self.scale_factor = scale_factor
        self.rng = np.random.RandomState(seed)
        self.length_data = None
        if sketches is None:
            cache = os.path.join(data_dir, data_filename + ".npz")
            if not os.path.exists(cache):
                raw_dir = os.path.join(data_dir, data_filename)
                print("creating training data cache from raw source " + raw_dir)
                _, self.length_data = preprocess(raw_dir, cache)
            sketches = load_stroke_cache(cache)
        # scale here rather than at construction (reference utils.py:219-225)
        self.raw_data = [np.array(s, dtype=np.float32, copy=True) for s in sketches]
        for s in self.raw_data:
            s[:, 0:2] /= self.scale_factor
        if not self.raw_data:
            raise ValueError("empty dataset")
        self.num_samples = len(self.raw_data)
        self.rank, self.world_size = rank, world_size
        self._flat = None
        self._offsets = None
        self._native = None
        if use_native:
            from ..utils import native
            self._native = native.host_lib()
        self.index = np.arange(self.num_samples)
        self.reset_index_pointer()

    # -- epoch bookkeeping ----------------------------------------------------------
    @property
    def pointer(self) -> int:
        return self._cursor.pointer

    @property
    def epoch_finished(self) -> bool:
        return self._cursor.epoch_finished

    def reset_index_pointer(self):
        # the reference re-shuffles the previous permutation (utils.py:279-283)
        self.index = self.rng.permutation(self.index)
        perm = self.index[self.rank::self.world_size] if self.world_size > 1 else self.index
        self._perm = np.ascontiguousarray(perm, dtype=np.int64)
        self._cursor = _Cursor(len(self._perm))

    def state_dict(self) -> dict:
        """JSON-serialisable cursor + RNG state (exact resume mid-epoch)."""
        name, keys, pos, has_g, g = self.rng.get_state()
        return {"rng": [name, keys.tolist(), int(pos), int(has_g), float(g)], "index": self.index.tolist(),
                "pointer": int(self._cursor.pointer), "epoch_finished": bool(self._cursor.epoch_finished)}

    def load_state_dict(self, sd: dict) -> None:
        name, keys, pos, has_g, g = sd["rng"]
        self.rng.set_state((name, np.asarray(keys, dtype=np.uint32), pos, has_g, g))
        self.index = np.asarray(sd["index"], dtype=np.int64)
        perm = self.index[self.rank::self.world_size] if self.world_size > 1 else self.index
        self._perm = np.ascontiguousarray(perm, dtype=np.int64)
        self._cursor = _Cursor(len(self._perm))
        self._cursor.pointer = int(sd["pointer"])
        self._cursor.epoch_finished = bool(sd["epoch_finished"])

    def current_data(self) -> np.ndarray:
        return self.raw_data[self._perm[self._cursor.pointer]]

    def tick_index_pointer(self):
        self._cursor.tick()

    # -- batching -----------------------------------------------------------------------
    def _flat_buffers(self):
        if self._flat is None:
            off = np.zeros(self.num_samples + 1, dtype=np.int64)
            for k, s in enumerate(self.raw_data):
                off[k + 1] = off[k] + len(s)
            self._flat = np.ascontiguousarray(np.concatenate(self.raw_data, 0), dtype=np.float32)
            self._offsets = off
        return self._flat, self._offsets

    def next_batch_full(self) -> np.ndarray:
        n = self.seq_length + 1
        scales = self.rng.rand(self.batch_size, 2) * 0.6 + 0.7
        if self._native is not None:
            flat, off = self._flat_buffers()
            out = np.zeros((self.batch_size, n, 5), dtype=np.float32)
            ptr, fin = self._native.pack_reference(flat, off, self._perm, self._cursor.pointer,
                                                   self._cursor.epoch_finished, self.batch_size, n,
                                                   np.ascontiguousarray(scales, dtype=np.float64), out)
            self._cursor.pointer, self._cursor.epoch_finished = ptr, fin
            return out
        return pack_rows_reference(self.raw_data, self._perm, self._cursor, self.batch_size, n, scales)

    def next_batch(self):
        batch = self.next_batch_full()
        return batch[:, 0:-1], batch[:, 1:]
