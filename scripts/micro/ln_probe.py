#!/usr/bin/env python3
"""Timing probe of the chained LayerNorm-LSTM steps (csrc/chain_step.hip
chain_ln_fwd / chain_ln_bwd at the vae_layernorm decoder shape: H = 512,
B = 100): forward + backward of one sequence repeated with
skr_chain_ln_set_probe(P) -- 0 the full launches, 1 producers only (the rows
end at once), 2 rows only (the producers only arrive). Run each P under
rocprofv3 --kernel-trace --stats; outputs are wrong while a probe is set.
usage: ln_probe.py P [reps]"""
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.utils import native  # noqa: E402


def main():
    probe = int(sys.argv[1])
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    torch.manual_seed(0)
    T, B, H = 30, 100, 512
    xp = torch.randn(T, B, 4 * H, device="cuda", requires_grad=True)
    W = (torch.randn(H, 4 * H, device="cuda") / math.sqrt(H)).requires_grad_()
    h0 = torch.zeros(B, H, device="cuda")
    ln = [torch.ones(4 * H, device="cuda", requires_grad=True), torch.zeros(4 * H, device="cuda", requires_grad=True),
          torch.ones(H, device="cuda", requires_grad=True), torch.zeros(H, device="cuda", requires_grad=True)]
    seed = torch.tensor([3], device="cuda")
    w = torch.randn(T, B, H, device="cuda")

    def run():
        out, _ = ops.lstm_sequence(xp, W, h0, h0, drop_keep=0.9, drop_seed=seed, drop_stream=4, ln=tuple(ln))
        torch.autograd.grad((out * w).sum(), [xp, W] + ln)

    lib = native.require_hip().lib
    run()
    torch.cuda.synchronize()
    prev = lib.skr_chain_ln_set_probe(probe)
    try:
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
    finally:
        lib.skr_chain_ln_set_probe(prev)
    print("probe %d: %d forward + backward passes of T = %d" % (probe, reps, T), flush=True)


if __name__ == "__main__":
    main()
