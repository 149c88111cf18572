#!/usr/bin/env python3
"""Per-phase view of REPLAYED optimizer steps in a rocprofv3 kernel trace.

A step is the span between two consecutive ``adam_kernel`` dispatches. The
trainer runs two eager warm-up steps inside GraphedStep before it captures,
so only the last ``--last N`` steps (default 1) are taken; call bench.py with
at least N + 1 timed steps after its warm-up so every selected step is a
graph replay. Loop kernels (recurrent GEMM / cell) are collapsed into one
line per loop; everything else is listed in launch order with its duration
(first selected step), and the per-kernel table averages the N steps.

usage: python scripts/prof_step.py <run_kernel_trace.csv> [min_us] [--last N]"""
import csv
import sys

LOOP = ("cell_fwd", "cell_bwd", "skinny_gemm", "lstm_fused", "chain_bwd", "hyper_mod_fwd")


def main():
    argv = [a for a in sys.argv[1:] if not a.startswith("--last")]
    last = 1
    for i, a in enumerate(sys.argv):
        if a.startswith("--last"):
            last = int(a.split("=")[1]) if "=" in a else int(sys.argv[i + 1])
            if "=" not in a:
                argv.remove(sys.argv[i + 1])
    rows = list(csv.DictReader(open(argv[0])))
    min_us = float(argv[1]) if len(argv) > 1 else 15.0
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    assert len(idx) > last, "need %d steps after a first optimizer step, trace has %d" % (last, len(idx))
    steps = [rows[idx[-k - 1] + 1: idx[-k] + 1] for k in range(last, 0, -1)]
    spans = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3 for s in steps]
    busy = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s) / 1e3 for s in steps]
    print("steps averaged: %d (the last %d of %d optimizer steps in the trace)" % (last, last, len(idx)))
    print("step span (first kernel start -> adam end) ms: %s; mean %.3f" % (
        " ".join("%.3f" % (x / 1e3) for x in spans), sum(spans) / len(spans) / 1e3))
    print("kernel busy time per step ms: mean %.3f" % (sum(busy) / len(busy) / 1e3))
    seq = steps[0]
    t0 = int(seq[0]["Start_Timestamp"])
    loop_start = loop_n = 0
    loop_sum = other = 0.0
    print("\nlaunch order, first selected step (kernels >= %.0f us; loops collapsed):" % min_us)
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
    print("non-loop kernels %.2f ms" % (other / 1e3))
    # per-kernel totals per step (duration = start-to-end of each dispatch;
    # concurrent streams overlap, so the sum can exceed the span)
    agg = {}
    for s in steps:
        for r in s:
            n = r["Kernel_Name"][:110]
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            a = agg.setdefault(n, [0, 0.0])
            a[0] += 1
            a[1] += d
    print("\nper kernel, mean per step over %d step(s):" % last)
    for n, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        print("%9.1f us %7.1f x %7.2f us  %s" % (d / last, c / last, d / c, n))
    # glue: PyTorch's own kernels, runtime copies / fills and library GEMMs
    # on the step (everything not hand-written in csrc/)
    kinds = (("at::native", "PyTorch elementwise / reduce / fill / cat"), ("rocclr", "runtime copy / fill"),
             ("Cijk_", "library GEMM"))
    print("\nglue per step (kernel time, mean over %d step(s)):" % last)
    tot = 0.0
    for key, what in kinds:
        c = sum(v[0] for n, v in agg.items() if key in n) / last
        d = sum(v[1] for n, v in agg.items() if key in n) / last
        tot += d
        print("%9.1f us %7.1f x  %s (%s)" % (d, c, what, key))
    print("%9.1f us total" % tot)


if __name__ == "__main__":
    main()
