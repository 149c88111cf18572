#!/usr/bin/env python3
"""Wide-decode knobs A/B on GraphDecoder decode steps of the vae_large
decoder (random init, early exit off), alternating settings:
ops.hyper.HM_ZGRID (0 = one workgroup per row block of the modulation
launch, k = k workgroups per tile walking the blocks) and
sample.hyper_step.WIDE_MAIN_C (main-cell workgroups per row above 128 rows).
One JSON line per (batch, setting, round)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.config import PRESETS  # noqa: E402
from sketch_rnn_amd.models.vae import SketchVAE  # noqa: E402
from sketch_rnn_amd.ops import hyper  # noqa: E402
from sketch_rnn_amd.sample import hyper_step  # noqa: E402
from sketch_rnn_amd.sample.sampler import GraphDecoder  # noqa: E402


def main():
    ops.set_backend("hip")
    ops.set_compute_dtype("bf16")
    cfg = PRESETS["vae_large"]
    m = SketchVAE(cfg, seed=0).cuda().eval()
    for B in (512, 1024):
        for rnd in range(2):
            for zg, mc in ((0, 1), (1, 1), (2, 1), (4, 1), (0, 2), (0, 4), (0, 8)):
                hyper.HM_ZGRID, hyper_step.WIDE_MAIN_C = zg, mc
                d = GraphDecoder(m, B, 250, 0.5, early_exit=False)
                d.run(seed=0)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                d.run(seed=1)
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                print(json.dumps({"batch": B, "zgrid": zg, "wide_main_c": mc, "round": rnd, "ms_per_decode_step": round(1000 * dt / d.steps_run, 4),
                                  "decode_positions_per_s": round(B * d.steps_run / dt, 1)}), flush=True)
                del d
    hyper.HM_ZGRID, hyper_step.WIDE_MAIN_C = 0, 1


if __name__ == "__main__":
    main()
