#!/usr/bin/env python3
"""Summary (mean / std of the final test recon NLL per arm, gap to the fp32
arm in units of its seed spread) over every per-seed line of one or more
scripts/converge.py JSONL files -- runs split over several GPU calls."""
import json
import sys

import numpy as np


def main():
    runs = []
    for path in sys.argv[1:]:
        with open(path) as f:
            for line in f:
                r = json.loads(line)
                if not r.get("summary"):
                    runs.append(r)
    arms = sorted({r["arm"] for r in runs})
    # commit: a tree identity dict (utils/provenance.py) or an older string label
    ident = lambda c: json.dumps(c, sort_keys=True) if isinstance(c, dict) else str(c)  # noqa: E731
    summ = {"summary": True, "commits": [json.loads(c) if c.startswith("{") else c
                                         for c in sorted({ident(r.get("commit", "unknown")) for r in runs})],
            "config": runs[0]["config"], "steps": runs[0]["steps"],
            "seeds": sorted({r["seed"] for r in runs}), "arms": {}}
    for a in arms:
        v = np.array([r["final_test_recon_nll"] for r in sorted(runs, key=lambda r: r["seed"]) if r["arm"] == a])
        summ["arms"][a] = {"mean": round(float(v.mean()), 5), "std": round(float(v.std(ddof=1)) if len(v) > 1 else 0.0, 5),
                           "finals": [float(x) for x in v],
                           "skipped_steps": [r.get("skipped_steps") for r in runs if r["arm"] == a]}
    ref = next((a for a in arms if a.endswith("fp32")), None)
    if ref is not None:
        m0 = summ["arms"][ref]["mean"]
        for a in arms:
            if a != ref:
                d = summ["arms"][a]["mean"] - m0
                summ["arms"][a]["rel_gap_vs_%s" % ref] = round(d / abs(m0), 5)
                summ["arms"][a]["gap_in_%s_std" % ref] = round(d / max(summ["arms"][ref]["std"], 1e-12), 3)
                summ["arms"][a]["within_1_std"] = bool(abs(d) <= summ["arms"][ref]["std"])
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
