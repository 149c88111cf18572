#!/usr/bin/env python3
"""Training-step A/B on one box: vae_large bench.py with the fused MDN head
reading the decoder's bf16 h rows (dW on the long-K weight-gradient GEMM) vs
the fp32 rows (row-slab dW kernel), alternated A B A B."""
import gc
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

import bench  # noqa: E402
from sketch_rnn_amd.ops import mdn_hip  # noqa: E402

steps = sys.argv[1] if len(sys.argv) > 1 else "20"
orig = mdn_hip._lp_rows
for rep in range(int(os.environ.get("AB_REPS", "2"))):
    for arm in ("bf16_rows", "fp32_rows"):
        mdn_hip._lp_rows = orig if arm == "bf16_rows" else (lambda X_lp, X, Hd: None)
        sys.argv = ["bench.py", "--steps", steps, "--warmup", "3", "--no-eval"]
        print("arm head=%s rep %d" % (arm, rep), flush=True)
        bench.main()
        gc.collect()
        torch.cuda.empty_cache()
mdn_hip._lp_rows = orig
