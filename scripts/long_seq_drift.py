"""Error growth of the HyperLSTM decoder over a long sequence (diagnostic).

Per time step, the max |difference| of the layer output between:
  hip-bf16 vs torch-fp32, hip-fp32 vs torch-fp32, and torch-fp32 vs
  torch-fp32 with the input perturbed by 1e-6 (the recurrence's own
  sensitivity: a chaotic trajectory amplifies any rounding the same way)."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.models import cells as C  # noqa: E402


def main():
    T, B, IN, Z, H, Hh, E = int(os.environ.get("LT", "250")), 8, 5, 16, 2048, 256, 32
    dev = torch.device("cuda")
    torch.manual_seed(8)
    p = C.HyperLSTMParams(IN + Z, H, Hh, E).to(dev)
    jit = float(os.environ.get("LJIT", "0"))
    with torch.no_grad():
        for prm in p.parameters():
            prm.add_(torch.randn_like(prm) * jit)
    x = torch.randn(T, B, IN, device=dev)
    z = torch.randn(B, Z, device=dev)
    st = [torch.zeros(B, n, device=dev) for n in (H, H, Hh, Hh)]

    def run(backend, dt, xx):
        ops.set_backend(backend)
        ops.set_compute_dtype(dt)
        with torch.no_grad():
            out, _ = ops.hyper_sequence(p, xx, *st, drop_keep=1.0, zc=z)
        return out.float()

    ref = run("torch", "fp32", x)
    res = {"bf16": run("hip", "bf16", x), "hip_fp32": run("hip", "fp32", x),
           "torch_perturbed": run("torch", "fp32", x + 1e-6 * torch.randn_like(x))}
    for k, v in res.items():
        d = (v - ref).abs().amax(dim=(1, 2))
        pts = [0, 1, 2, 5, 10, 20, 50, 100, 150, 200, T - 1]
        print(json.dumps({"vs_torch_fp32": k, "max_abs_err_at_t": {t: round(float(d[t]), 5) for t in pts if t < T},
                          "ref_max": round(float(ref.abs().max()), 4)}), flush=True)


if __name__ == "__main__":
    main()
