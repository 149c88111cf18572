#!/usr/bin/env python3
"""Training-step A/B on one box: vae_large bench.py with the round-5 weight
gradient schedule (fragment reads of both k16 halves up front, dP at 5
splits) vs the round-4 one (per-half reads, dP at 2 splits), alternated
A B A B so clock / box drift hits both arms alike."""
import gc
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

import bench  # noqa: E402
from sketch_rnn_amd.ops import gemm  # noqa: E402
from sketch_rnn_amd.utils import native  # noqa: E402

steps = sys.argv[1] if len(sys.argv) > 1 else "20"
lib = native.require_hip().lib
for rep in range(int(os.environ.get("AB_REPS", "2"))):
    for arm in ("r5", "r4"):
        lib.skr_wgrad_set_variant(1 if arm == "r5" else 0)
        gemm.WGRAD_SPLIT = {} if arm == "r5" else {(256, 24576, 1): 2}
        sys.argv = ["bench.py", "--steps", steps, "--warmup", "3", "--no-eval"]
        print("arm wgrad=%s rep %d" % (arm, rep), flush=True)
        bench.main()
        gc.collect()
        torch.cuda.empty_cache()
