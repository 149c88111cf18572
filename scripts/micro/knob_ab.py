#!/usr/bin/env python3
"""Training-step A/B on one box over module-attribute knobs: each arm is a
comma-separated list of ``module.ATTR=value`` settings (module relative to
``sketch_rnn_amd.ops``, value a Python literal); arms are alternated
A B C A B C ... so clock / box drift hits every arm alike. Each arm runs
bench.py in this process (same HIP library, fresh trainer + graph).

usage: knob_ab.py [--steps N] [--reps R] [--bench "extra bench args"] ARM [ARM ...]
  e.g. knob_ab.py --steps 20 "hyper.BG_WGRAD=False" "hyper.BG_WGRAD=True,hyper.BG_GRID=32"
"""
import ast
import gc
import importlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

import bench  # noqa: E402


def parse_arm(spec):
    import re
    out = []
    # items split at commas that start a new "module.ATTR=" (values may hold commas)
    for item in filter(None, re.split(r",(?=\s*[A-Za-z_][\w.]*\.[A-Za-z_]\w*\s*=)", spec)):
        key, val = item.split("=", 1)
        mod, attr = key.rsplit(".", 1)
        out.append((importlib.import_module("sketch_rnn_amd.ops." + mod), attr, ast.literal_eval(val)))
    return out


def main():
    args = sys.argv[1:]
    steps, reps, extra = "20", 2, []
    while args and args[0].startswith("--"):
        flag = args.pop(0)
        if flag == "--steps":
            steps = args.pop(0)
        elif flag == "--reps":
            reps = int(args.pop(0))
        elif flag == "--bench":
            extra = args.pop(0).split()
    arms = [(spec, parse_arm(spec)) for spec in args]
    defaults = {(id(m), a): getattr(m, a) for _, arm in arms for m, a, _ in arm}
    for rep in range(reps):
        for spec, arm in arms:
            for _spec, other in arms:   # every knob back to its default, then this arm's settings
                for m, a, _v in other:
                    setattr(m, a, defaults[(id(m), a)])
            for m, a, v in arm:
                setattr(m, a, v)
            sys.argv = ["bench.py", "--steps", steps, "--warmup", "3", "--no-eval"] + extra
            print("arm %s rep %d" % (spec, rep), flush=True)
            bench.main()
            gc.collect()
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
