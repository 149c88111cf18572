"""Tracing and per-phase timing.

* :func:`phase` -- a named range: a roctx range (``torch.cuda.nvtx`` maps to
  roctx on ROCm, so ``rocprofv3 --marker-trace`` shows it) plus optional
  host wall time into a :class:`PhaseTimes` accumulator.
* :class:`GpuPhaseTimer` -- hipEvent pairs around GPU work (forward/backward
  graph, all-reduce, optimizer) read back once per log interval, so timing
  never adds a sync inside the step.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import torch

_ENABLED = True


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


class PhaseTimes:
    """Host wall-clock seconds per phase name (summed)."""

    def __init__(self):
        self.total: Dict[str, float] = defaultdict(float)
        self.count: Dict[str, int] = defaultdict(int)

    def add(self, name: str, dt: float) -> None:
        self.total[name] += dt
        self.count[name] += 1

    def mean_ms(self) -> Dict[str, float]:
        return {k: 1000.0 * v / max(self.count[k], 1) for k, v in self.total.items()}

    def reset(self) -> None:
        self.total.clear()
        self.count.clear()


@contextlib.contextmanager
def phase(name: str, times: Optional[PhaseTimes] = None):
    marked = _ENABLED and torch.cuda.is_available()
    if marked:
        torch.cuda.nvtx.range_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if times is not None:
            times.add(name, time.perf_counter() - t0)
        if marked:
            torch.cuda.nvtx.range_pop()


class GpuPhaseTimer:
    """Records (start, end) hipEvents per named phase on the current stream;
    :meth:`collect` synchronises once and returns mean milliseconds."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self._open: Dict[str, torch.cuda.Event] = {}
        self._done: List[Tuple[str, torch.cuda.Event, torch.cuda.Event]] = []

    def start(self, name: str) -> None:
        if self.enabled:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._open[name] = e

    def stop(self, name: str) -> None:
        if self.enabled and name in self._open:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._done.append((name, self._open.pop(name), e))

    @contextlib.contextmanager
    def time(self, name: str):
        self.start(name)
        try:
            yield
        finally:
            self.stop(name)

    def collect(self) -> Dict[str, float]:
        if not self._done:
            return {}
        self._done[-1][2].synchronize()
        acc: Dict[str, List[float]] = defaultdict(list)
        for name, a, b in self._done:
            acc[name].append(a.elapsed_time(b))
        self._done.clear()
        return {k: sum(v) / len(v) for k, v in acc.items()}
