#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: time per training step by kernel.

usage: prof_summary.py run_kernel_stats.csv [steps] [top N] [--per-kernel NAME]

``steps`` is the number of training steps the trace covers. When omitted it
is inferred from the number of calls of the optimizer kernel (``adam_kernel``
runs exactly once per training step) so that "ms/step" really is per step.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    steps = float(sys.argv[2]) if len(sys.argv) > 2 and float(sys.argv[2]) > 0 else 0.0
    if steps == 0.0:
        adam = [int(r["Calls"]) for r in rows if "adam_kernel" in r["Name"]]
        steps = float(adam[0]) if adam else 1.0
        how = "inferred from adam_kernel calls" if adam else "no adam_kernel: totals"
    else:
        how = "given"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("traced steps: %d (%s); kernel time total %.2f ms, per step %.3f ms"
          % (steps, how, tot / 1e6, tot / 1e6 / steps))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print("%8.3f ms/step %7.1f calls/step %8.2f us avg  %s" % (
            float(r["TotalDurationNs"]) / 1e6 / steps, int(r["Calls"]) / steps, float(r["AverageNs"]) / 1e3,
            r["Name"][:100]))


if __name__ == "__main__":
    main()
