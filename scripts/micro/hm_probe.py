#!/usr/bin/env python3
"""Timing probe of the training modulation step (csrc/hyper_mod.hip
hyper_mod_fwd at the vae_large shape: B = 100, H = 2048, Hh = 256): the
HyperLSTM forward (training kernels, no backward) repeated with
skr_hyper_mod_set_probe(P) -- 0 the full kernel, 1 dispatch + P fragments,
2 + every load and the hh LDS stage, 3 + the MFMAs (no vector stage,
epilogue or stores), 4 dispatch only. Run each P under rocprofv3 --kernel-trace --stats and
read hyper_mod_fwd's mean duration; outputs are wrong while a probe is set.
usage: hm_probe.py P [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.models import cells as C  # noqa: E402
from sketch_rnn_amd.utils import native  # noqa: E402


def main():
    probe = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    torch.manual_seed(0)
    T, B, IN, Z, H, Hh, E = 30, 100, 5, 128, 2048, 256, 32
    p = C.HyperLSTMParams(IN + Z, H, Hh, E).to("cuda")
    x = torch.randn(T, B, IN, device="cuda")
    z = torch.randn(B, Z, device="cuda", requires_grad=True)
    st = [torch.zeros(B, n, device="cuda") for n in (H, H, Hh, Hh)]
    lib = native.require_hip().lib
    ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=1, drop_stream=9, zc=z)   # setup (weight caches)
    torch.cuda.synchronize()
    prev = lib.skr_hyper_mod_set_probe(probe)
    try:
        for _ in range(reps):
            ops.hyper_sequence(p, x, *st, drop_keep=0.9, drop_seed=1, drop_stream=9, zc=z)
        torch.cuda.synchronize()
    finally:
        lib.skr_hyper_mod_set_probe(prev)
    print("probe %d: %d forward passes of T = %d" % (probe, reps, T), flush=True)


if __name__ == "__main__":
    main()
