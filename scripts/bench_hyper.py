"""HyperLSTM decoder scan at the vae_large shape (H 2048, Hh 256, E 32,
B 100, T 250, bf16): forward-only and forward+backward time of the
per-step launch chain, replayed from a HIP graph. One JSON line."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.models import cells as C  # noqa: E402
from sketch_rnn_amd.ops import recurrent  # noqa: E402  (check_cluster_errors)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=250)
    ap.add_argument("--B", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda")
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    torch.manual_seed(0)
    T, B, IN, Z, H, Hh, E = args.T, args.B, 5, 128, 2048, 256, 32
    p = C.HyperLSTMParams(IN + Z, H, Hh, E).to(dev)
    x = torch.randn(T, B, IN, device=dev)
    z = torch.randn(B, Z, device=dev, requires_grad=True)
    st = [torch.zeros(B, n, device=dev) for n in (H, H, Hh, Hh)]
    w = torch.randn(T, B, H, device=dev)
    for var in ("chain",):
        res = {"variant": var, "T": T, "B": B}
        for mode in ("fwd", "fwdbwd"):
            def step():
                if mode == "fwd":
                    with torch.no_grad():
                        out, _ = ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=1, drop_stream=9, zc=z)
                    return out
                out, _ = ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=1, drop_stream=9, zc=z)
                return torch.autograd.grad((out * w).sum(), [z] + list(p.parameters()))
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                step()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[mode + "_ms"] = round(e0.elapsed_time(e1) / args.reps, 3)
            del g
        recurrent.check_cluster_errors(dev)
        res["fwd_us_per_step"] = round(1000 * res["fwd_ms"] / T, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
