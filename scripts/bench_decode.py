#!/usr/bin/env python3
"""Decode throughput of the reference model (2 x 256 LSTM, M = 24, T = 300
strokes per sketch): the fused whole-sketch kernel (FusedRefDecoder, one
launch per batch) against the HIP-graph decoder (GraphDecoder: per-stroke
kernel chain replayed from one graph), both with the on-device sampler and
bf16 operands. Prints one JSON line per (impl, batch)."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.config import RefConfig  # noqa: E402
from sketch_rnn_amd.models.reference import SketchRNN  # noqa: E402
from sketch_rnn_amd.sample.fused import FusedRefDecoder  # noqa: E402
from sketch_rnn_amd.sample.sampler import GraphDecoder  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--batches", default="1,16,64,224")
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    m = SketchRNN(RefConfig(), seed=0).to("cuda").eval()
    for B in [int(b) for b in a.batches.split(",")]:
        for impl in ("fused", "graph"):
            dec = (FusedRefDecoder(m, B, a.steps, temperature=0.5) if impl == "fused"
                   else GraphDecoder(m, B, a.steps, temperature=0.5))
            s = timed(lambda: dec.run(seed=1), a.reps)
            print(json.dumps({"bench": "reference decode", "impl": impl, "batch": B, "steps": a.steps,
                              "ms_per_batch": round(s * 1e3, 3), "us_per_step": round(s * 1e6 / a.steps, 2),
                              "strokes_per_s": round(B * a.steps / s, 1)}), flush=True)


if __name__ == "__main__":
    main()
