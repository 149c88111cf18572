#!/usr/bin/env python3
"""Training-step A/B on one box: vae_large bench.py with the HyperLSTM main
input projection stored in bf16 (sketch_rnn_amd.ops.hyper.XH_BF16) vs fp32,
alternated A B A B so clock / box drift hits both arms alike."""
import gc
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

import bench  # noqa: E402
from sketch_rnn_amd.ops import hyper  # noqa: E402

steps = sys.argv[1] if len(sys.argv) > 1 else "20"
for rep in range(int(os.environ.get("AB_REPS", "2"))):
    for arm in (True, False):
        hyper.XH_BF16 = arm
        sys.argv = ["bench.py", "--steps", steps, "--warmup", "3", "--no-eval"]
        print("arm xh_bf16=%s rep %d" % (arm, rep), flush=True)
        bench.main()
        gc.collect()
        torch.cuda.empty_cache()
