"""Per-kernel launch floor on the GPU: a chain of N dependent tiny kernels,
eager and replayed from a HIP graph (torch.cuda.graph), timed with events.

Prints one JSON line per mode: microseconds per kernel. Used to price the
kernel boundary of the per-step recurrent launch chains (env knobs such as
HIP_FORCE_DEV_KERNARG are read by the HIP runtime at process start, so run
one process per setting)."""
from __future__ import annotations

import argparse
import json
import os

import torch


def chain(x, n):
    for _ in range(n):
        x.add_(1.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--numel", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    x = torch.zeros(args.numel, device=dev)
    res = {"env": {k: os.environ.get(k) for k in ("HIP_FORCE_DEV_KERNARG", "DEBUG_CLR_GRAPH_PACKET_CAPTURE",
                                                  "GPU_MAX_HW_QUEUES")}, "numel": args.numel}
    # eager
    chain(x, 50)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(args.reps):
        chain(x, args.n)
    e.record()
    torch.cuda.synchronize()
    res["eager_us_per_kernel"] = s.elapsed_time(e) * 1000 / (args.reps * args.n)
    # graph
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        chain(x, 10)
    torch.cuda.current_stream().wait_stream(st)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        chain(x, args.n)
    g.replay()
    torch.cuda.synchronize()
    s.record()
    for _ in range(args.reps):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    res["graph_us_per_kernel"] = s.elapsed_time(e) * 1000 / (args.reps * args.n)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
