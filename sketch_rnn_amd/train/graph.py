"""HIP-graph capture of a whole training step (forward + backward + optimizer).

On MI355X a recurrent training step is thousands of small dependent kernels
(per time step: recurrent GEMM + fused cell kernel, forward and reverse).
Replaying them from one captured ``hipGraph`` removes the per-launch host
cost and the inter-kernel host gaps; this is the framework's replacement
for a tracing compiler.

Contract for a capturable step function ``fn(**static)``:
* reads only from the static input tensors (refreshed by ``copy_`` before
  each replay) and from device-resident state (weights, optimizer arena,
  the dropout seed tensor, the lr scalar);
* performs no host synchronisation and no allocation that depends on data.

Warm-up runs needed before capture mutate the training state, so
:class:`GraphedStep` snapshots the optimizer arena (weights, moments,
scalars) and restores it after capture.
"""
from __future__ import annotations

import contextlib
import gc
from typing import Callable, Dict, Optional

import torch


@contextlib.contextmanager
def capture(graph: "torch.cuda.CUDAGraph", pool=None):
    """``torch.cuda.graph`` with Python's cyclic GC held off for the
    duration of the capture. A collection triggered by an allocation inside
    the captured region could run the destructor of an unreachable object
    that owns HIP resources (an earlier ``CUDAGraph``, an event), and such
    HIP calls are illegal while a stream is capturing -- the process aborts.
    Garbage is collected before the capture instead. Under an initialised
    process group the capture mode is "thread_local": the RCCL watchdog
    thread polls collective events concurrently and must not invalidate it."""
    import torch.distributed as dist
    mode = "thread_local" if dist.is_available() and dist.is_initialized() else "global"
    gc.collect()
    enabled = gc.isenabled()
    gc.disable()
    try:
        with torch.cuda.graph(graph, pool=pool, capture_error_mode=mode):
            yield
    finally:
        if enabled:
            gc.enable()


class GraphedStep:
    def __init__(self, fn: Callable[..., Dict[str, torch.Tensor]], static_inputs: Dict[str, torch.Tensor],
                 warmup: int = 2, snapshot: Optional[list] = None):
        self.fn = fn
        self.static = static_inputs
        saved = [t.detach().clone() for t in (snapshot or [])]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                fn(**self.static)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with capture(self.graph):
            self.outputs = fn(**self.static)
        torch.cuda.synchronize()
        with torch.no_grad():
            for t, s in zip(snapshot or [], saved):
                t.copy_(s)

    def __call__(self, **inputs) -> Dict[str, torch.Tensor]:
        for k, v in inputs.items():
            dst = self.static[k]
            if v.data_ptr() != dst.data_ptr():
                dst.copy_(v, non_blocking=True)
        self.graph.replay()
        return self.outputs


class GraphedPhases:
    """A step split into consecutive phases, each captured in its own HIP
    graph (one shared memory pool, replayed in capture order), so that host
    work -- the RCCL collectives of data parallelism -- can be issued
    between them while the next phase runs.

    ``phases[0]`` takes the static inputs; later phases take no arguments
    and communicate through state they keep themselves (e.g. the encoder
    outputs and their gradients stashed by phase 0 for phase 1). Warm-up
    runs every phase in order; the optimizer arena is snapshotted and
    restored around warm-up + capture exactly as in :class:`GraphedStep`.
    """

    def __init__(self, phases, static_inputs: Dict[str, torch.Tensor], warmup: int = 2,
                 snapshot: Optional[list] = None):
        self.phases = list(phases)
        self.static = static_inputs
        saved = [t.detach().clone() for t in (snapshot or [])]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                self.phases[0](**self.static)
                for fn in self.phases[1:]:
                    fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graphs = []
        self.outputs = []
        pool = None
        for i, fn in enumerate(self.phases):
            g = torch.cuda.CUDAGraph()
            with capture(g, pool=pool):
                self.outputs.append(fn(**self.static) if i == 0 else fn())
            pool = g.pool() if pool is None else pool
            self.graphs.append(g)
        torch.cuda.synchronize()
        with torch.no_grad():
            for t, s in zip(snapshot or [], saved):
                t.copy_(s)

    def replay(self, i: int, **inputs):
        if i == 0:
            for k, v in inputs.items():
                dst = self.static[k]
                if v.data_ptr() != dst.data_ptr():
                    dst.copy_(v, non_blocking=True)
        self.graphs[i].replay()
        return self.outputs[i]
