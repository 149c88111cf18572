"""Background batch producer for the training loop.

Building a VAE batch (random scaling, point-drop augmentation, padding to
``Nmax``) is ~1 ms of NumPy per 100 sketches -- host time that would sit
between two HIP-graph replays. :class:`Prefetcher` runs it on one daemon
thread ``depth`` batches ahead and stages each batch in page-locked host
tensors, so the trainer's host->device copy is an async DMA on the compute
stream and the GPU never waits for the data pipeline.

Exact resume: the thread is the only consumer of the dataset's RNGs and it
records the dataset state right after producing each batch; the trainer
checkpoints the state attached to the last batch it *consumed*, so batches
sitting in the queue are regenerated after a restart instead of skipped.
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, Optional

import numpy as np
import torch


class Prefetcher:
    def __init__(self, produce: Callable[[], tuple], state: Optional[Callable[[], dict]] = None,
                 depth: int = 2, pin: bool = True):
        self._produce, self._state = produce, state
        self._q: "queue.Queue" = queue.Queue(maxsize=max(1, depth))
        self._stop = threading.Event()
        self._pin = pin and torch.cuda.is_available()
        self.consumed_state: Optional[dict] = None
        self._err: Optional[BaseException] = None
        self._t = threading.Thread(target=self._run, name="skr-prefetch", daemon=True)
        self._t.start()

    def _stage(self, a):
        t = torch.from_numpy(np.ascontiguousarray(a))
        return t.pin_memory() if self._pin else t

    def _run(self):
        try:
            while not self._stop.is_set():
                batch = tuple(self._stage(a) for a in self._produce())
                st = self._state() if self._state is not None else None
                while not self._stop.is_set():
                    try:
                        self._q.put((batch, st), timeout=0.1)
                        break
                    except queue.Full:
                        continue
        except BaseException as e:   # surfaced to the consumer on its next get()
            self._err = e
            self._q.put((None, None))

    def get(self):
        """Next batch (tuple of host tensors, pinned on a GPU machine)."""
        batch, st = self._q.get()
        if batch is None:
            raise RuntimeError("batch producer failed") from self._err
        self.consumed_state = st
        return batch

    def close(self):
        self._stop.set()
        try:
            while True:
                self._q.get_nowait()
        except queue.Empty:
            pass
        self._t.join(timeout=5)
