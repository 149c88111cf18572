#!/usr/bin/env python3
"""Per-phase view of the LAST optimizer step in a rocprofv3 kernel trace:
loop kernels (recurrent GEMM / cell) are collapsed into one line per loop,
everything else listed in launch order with its duration.
usage: python scripts/prof_step.py <run_kernel_trace.csv> [min_us]"""
import csv
import sys

LOOP = ("cell_fwd", "cell_bwd", "skinny_gemm", "lstm_fused")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 15.0
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    seq = rows[idx[-2] + 1: idx[-1] + 1]
    t0 = int(seq[0]["Start_Timestamp"])
    span = (int(seq[-1]["End_Timestamp"]) - t0) / 1e3
    loop_start = loop_n = 0
    loop_sum = other = 0.0
    for r in seq:
        n = r["Kernel_Name"]
        ts, d = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if any(k in n for k in LOOP):
            if loop_n == 0:
                loop_start = ts
            loop_n += 1
            loop_sum += d
            continue
        if loop_n:
            print("  [loop: %d kernels, %.0f us busy, %.0f us span]" % (loop_n, loop_sum, ts - loop_start))
            loop_n, loop_sum = 0, 0.0
        other += d
        if d >= min_us:
            print("%8.1f us  t=%8.0f  %s" % (d, ts, n[:100]))
    print("step span %.2f ms; non-loop kernels %.2f ms" % (span / 1e3, other / 1e3))
    # per-kernel totals inside the step (duration = start-to-end, which under
    # graph replay includes the kernel-boundary gap to the previous launch)
    agg = {}
    for r in seq:
        n = r["Kernel_Name"][:110]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += d
    print("\nper kernel (last step):")
    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
        print("%9.1f us %5d x %7.2f us  %s" % (d, c, d / c, n))


if __name__ == "__main__":
    main()
