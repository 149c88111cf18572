"""Padded, length-masked stroke-5 dataset for the seq2seq VAE.

Capability parity with the sketch-rnn VAE data pipeline that BASELINE.json
names (stroke-3 input, normalisation by the offset standard deviation,
random per-axis scaling, point-drop augmentation, S0 start token, padding
with end-of-sketch rows). Batches come out as ``float32`` arrays ready for a
single pinned host->device copy:

* ``strokes``  ``[B, Nmax + 1, 5]`` magenta stroke-5 with S0 at t=0;
* ``lengths``  ``[B]`` int64 number of real points;
* ``labels``   ``[B]`` int64 class id (class-conditional training).

DP sharding: ``random_batch(rank, world)`` draws one global permutation per
step from a seed shared by all ranks and takes the rank's contiguous slice,
so the union over ranks is exactly a single-process global batch.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from .strokes import augment_strokes, pad_batch_magenta, random_scale


class StrokeDataset:
    def __init__(self, strokes: Sequence[np.ndarray], batch_size: int = 100, max_seq_length: int = 250,
                 scale_factor: float = 1.0, random_scale_factor: float = 0.0, augment_stroke_prob: float = 0.0,
                 limit: float = 1000.0, labels: Optional[Sequence[int]] = None, seed: int = 0,
                 rank: int = 0):
        self.batch_size = batch_size
        self.max_seq_length = max_seq_length
        self.scale_factor = scale_factor
        self.random_scale_factor = random_scale_factor
        self.augment_stroke_prob = augment_stroke_prob
        self.limit = limit
        # batch selection is shared by all DP ranks; augmentation is per rank
        self.rng = np.random.RandomState(seed)
        self.aug_rng = np.random.RandomState(seed * 7919 + 1 + rank)
        kept, kept_labels, lens = [], [], []
        for k, s in enumerate(strokes):
            if len(s) <= max_seq_length:
                d = np.clip(np.asarray(s, dtype=np.float32), -limit, limit)
                d = np.array(d, dtype=np.float32, copy=True)
                d[:, 0:2] /= scale_factor
                kept.append(d)
                kept_labels.append(int(labels[k]) if labels is not None else 0)
                lens.append(len(d))
        order = np.argsort(np.asarray(lens), kind="stable")
        self.strokes: List[np.ndarray] = [kept[i] for i in order]
        self.labels = np.asarray([kept_labels[i] for i in order], dtype=np.int64)
        self.num_batches = len(self.strokes) // batch_size

    def __len__(self):
        return len(self.strokes)

    # -- normalisation -------------------------------------------------------------
    def calculate_normalizing_scale_factor(self) -> float:
        xy = np.concatenate([s[:, 0:2].reshape(-1) for s in self.strokes if len(s) <= self.max_seq_length])
        return float(np.std(xy))

    def normalize(self, scale_factor: Optional[float] = None) -> float:
        if scale_factor is None:
            scale_factor = self.calculate_normalizing_scale_factor()
        self.scale_factor = scale_factor
        for s in self.strokes:
            s[:, 0:2] /= scale_factor
        return scale_factor

    # -- resume ----------------------------------------------------------------------
    @staticmethod
    def _rng_state(r: np.random.RandomState):
        name, keys, pos, has_g, g = r.get_state()
        return [name, keys.tolist(), int(pos), int(has_g), float(g)]

    @staticmethod
    def _set_rng(r: np.random.RandomState, st):
        r.set_state((st[0], np.asarray(st[1], dtype=np.uint32), st[2], st[3], st[4]))

    def state_dict(self) -> dict:
        return {"rng": self._rng_state(self.rng), "aug_rng": self._rng_state(self.aug_rng)}

    def load_state_dict(self, sd: dict) -> None:
        self._set_rng(self.rng, sd["rng"])
        self._set_rng(self.aug_rng, sd["aug_rng"])

    # -- batching ------------------------------------------------------------------
    def _from_indices(self, indices, augment: bool = True):
        batch, lens = [], []
        for i in indices:
            d = self.strokes[i]
            if augment and self.random_scale_factor > 0:
                d = random_scale(d, self.random_scale_factor, self.aug_rng)
            else:
                d = np.array(d, copy=True)
            if augment and self.augment_stroke_prob > 0:
                d = augment_strokes(d, self.augment_stroke_prob, self.aug_rng)
            batch.append(d)
            lens.append(len(d))
        return pad_batch_magenta(batch, self.max_seq_length), np.asarray(lens, dtype=np.int64), \
            self.labels[np.asarray(list(indices), dtype=np.int64)]

    def random_batch(self, rank: int = 0, world: int = 1, batch_size: Optional[int] = None):
        """Per-rank slice of a global random batch of ``batch_size * world``."""
        b = batch_size or self.batch_size
        perm = self.rng.permutation(len(self.strokes))[: b * world]
        if len(perm) < b * world:
            perm = self.rng.randint(0, len(self.strokes), size=b * world)
        return self._from_indices(perm[rank * b:(rank + 1) * b])

    def get_batch(self, idx: int):
        assert 0 <= idx < self.num_batches
        start = idx * self.batch_size
        return self._from_indices(range(start, start + self.batch_size), augment=False)


def max_len(strokes: Sequence[np.ndarray]) -> int:
    return max((len(s) for s in strokes), default=0)
