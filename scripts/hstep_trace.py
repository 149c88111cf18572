"""Phase timeline of the fused HyperLSTM step kernels (diagnostic).

Needs the trace build: ``python scripts/build_native.py --variant trace_hstep``
and ``SKR_HIP_LIB=sketch_rnn_amd/_lib/variants/libskrnn_hip_trace_hstep.so``.
Runs one training forward + backward at the vae_large decoder geometry and
prints, per role of csrc/hyper_step.hip, the median / p90 / max of every
phase stamp (us from the launch's first workgroup start) of the last
forward launch and the last backward launch."""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.models import cells as C  # noqa: E402
from sketch_rnn_amd.utils import native  # noqa: E402


def summarize(buf, roles, labels):
    st = buf.cpu().numpy().astype(np.int64)
    t0 = st[st[:, 0] > 0, 0].min()
    out = {}
    for name, (lo, hi) in roles.items():
        blk = st[lo:hi]
        row = {}
        for k, lab in enumerate(labels[name]):
            v = blk[:, k]
            v = v[v > 0]
            if len(v) == 0:
                continue
            us = (v - t0) / 100.0
            row[lab] = [round(float(np.median(us)), 2), round(float(np.percentile(us, 90)), 2), round(float(us.max()), 2)]
        out[name] = row
    return out


def main():
    T, B, IN, Z, H, Hh, E = int(os.environ.get("LT", "12")), 100, 5, 128, 2048, 256, 32
    dev = torch.device("cuda")
    lib = native.require_hip()
    torch.manual_seed(1)
    p = C.HyperLSTMParams(IN + Z, H, Hh, E).to(dev)
    x = torch.randn(T, B, IN, device=dev)
    z = torch.randn(B, Z, device=dev, requires_grad=True)
    st = [torch.zeros(B, n, device=dev) for n in (H, H, Hh, Hh)]
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    buf = torch.zeros(2048, 8, dtype=torch.int64, device=dev)
    for rep in range(3):          # the last repetition is reported (warm caches)
        buf.zero_()
        assert lib.lib.skr_hstep_trace(ctypes_ptr(buf)) == 0
        out, _ = ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=3, drop_stream=9, zc=z)
        torch.cuda.synchronize()
        fwd = buf.clone()
        buf.zero_()
        (out * 0.01).sum().backward()
        torch.cuda.synchronize()
        bwd = buf.clone()
    lib.lib.skr_hstep_trace(None)
    S_y, S_h, S_am, S_ay = 4, 32, 8, 4
    nY, nR = (4 * Hh // 64) * S_y, 4 * H // 32
    f = summarize(fwd, {"rhyp": (0, nY), "hyper_row": (nY, nY + B), "main_tile": (nY + B, nY + B + nR)},
                  {"rhyp": ["start", "gemm", "arrive"], "hyper_row": ["start", "waited", "arrive"],
                   "main_tile": ["start", "gemm", "prefetched", "hh_ready", "z_done", "end"]})
    nV, nM, nYb = (Hh // 64) * S_h, (H // 64) * S_am, ((H + Hh) // 64) * S_ay
    b = summarize(bwd, {"dvec": (0, nV), "drm": (nV, nV + nM), "hyper_row": (nV + nM, nV + nM + B),
                        "dry": (nV + nM + B, nV + nM + B + nYb)},
                  {"dvec": ["start", "gemm", "arrive"], "drm": ["start", "gemm", "end"],
                   "hyper_row": ["start", "waited", "arrive"], "dry": ["start", "w_loaded", "waited", "end"]})
    print(json.dumps({"fwd_us": f}, indent=1))
    print(json.dumps({"bwd_us": b}, indent=1))


def ctypes_ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr())


if __name__ == "__main__":
    main()
