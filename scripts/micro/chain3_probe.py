#!/usr/bin/env python3
"""Where the three-stage chained backward launch spends its time
(csrc/chain_step.hip skr_chain_bwd_main3): HyperLSTM H 2048 forward +
backward (T steps, graph-replayed) for several batch sizes, per variant:

  chain2   two-stage chained launch + separate dvec P^T launch (default before)
  chain3   three-stage launch
  probe1   three-stage kernel, producers exit after their tile (no dvec P^T:
           isolates the rows' sc1 dvec stores + arrival)
  probe2   three-stage kernel, the tail stages its weights and waits on the
           rows, computes nothing
  probe3   three-stage kernel, the tail only waits on the rows (isolates
           holding the producers' CUs until the rows finish)

Probes 1/2 produce wrong gradients (timing only). One JSON line per (B, variant)
with the backward cost per time step."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.models import cells as C  # noqa: E402
from sketch_rnn_amd.ops import hyper  # noqa: E402
from sketch_rnn_amd.utils import native  # noqa: E402


def timed(fn, reps):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    lib = native.require_hip().lib
    dev = torch.device("cuda")
    print(json.dumps({"cus": torch.cuda.get_device_properties(0).multi_processor_count}), flush=True)
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    for B in (64, 100):
        torch.manual_seed(0)
        p = C.HyperLSTMParams(133, 2048, 256, 32).to(dev)
        x = torch.randn(T, B, 5, device=dev)
        z = torch.randn(B, 128, device=dev, requires_grad=True)
        st = [torch.zeros(B, n, device=dev) for n in (2048, 2048, 256, 256)]
        w = torch.randn(T, B, 2048, device=dev)

        def fwd():
            with torch.no_grad():
                ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=1, drop_stream=9, zc=z)

        def fwdbwd():
            out, _ = ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=1, drop_stream=9, zc=z)
            torch.autograd.grad((out * w).sum(), [z] + list(p.parameters()))
        f_ms = timed(fwd, 5)
        for var, c3, probe, poll in (("chain2", False, 0, 1), ("chain2_poll4", False, 0, 4),
                                     ("chain2_poll16", False, 0, 16), ("chain3", True, 0, 1),
                                     ("probe1", True, 1, 1), ("probe2", True, 2, 1), ("probe3", True, 3, 1)):
            hyper.CHAIN3 = c3
            lib.skr_chain3_set_probe(probe)
            lib.skr_chain_set_poll(poll)
            fb = timed(fwdbwd, 5)
            lib.skr_chain3_set_probe(0)
            lib.skr_chain_set_poll(1)
            print(json.dumps({"B": B, "T": T, "variant": var, "fwd_ms": round(f_ms, 3), "fwdbwd_ms": round(fb, 3),
                              "bwd_us_per_step": round(1000 * (fb - f_ms) / T, 2)}), flush=True)
    hyper.CHAIN3 = True


if __name__ == "__main__":
    main()
