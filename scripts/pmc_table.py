#!/usr/bin/env python3
"""Per-kernel memory traffic table from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE: kilobytes moved between L2 and memory, i.e.
HBM / MALL traffic, not L2 hits) plus the kernel-trace durations of a
separate non-counter run (counter passes serialise dispatches, so their own
timestamps overstate short kernels).

The reported counts are divided by the reported/true ratios of this box's
calibration run (profiles/r6/pmc_calibration.log: scripts/micro/pmc_calib
moves a known 1 GiB per launch; FETCH_SIZE read 0.500 of the true bytes for
16-B register loads, 8-B register loads and 16-B LDS-DMA loads alike, and
WRITE_SIZE 1.000 for 16-B and 8-B stores). Access widths the calibration did
not cover are corrected with the same ratios and marked as such in the
header; %peak is against the 8 TB/s datasheet HBM rate.

usage: pmc_table.py FETCH_counter_collection.csv WRITE_counter_collection.csv
                    [kernel_stats.csv] [top N] [--calib DIR]
"""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name
    for p in ("void ", "(anonymous namespace)::", "skr::"):
        n = n.replace(p, "")
    return n.split("(")[0].strip()[:70]


def read_counter(path):
    vals, dur, calls = defaultdict(float), defaultdict(float), defaultdict(int)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            vals[k] += float(r["Counter_Value"])
            calls[k] += 1
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    return vals, dur, calls


def _calib(path_dir):
    import json
    import os
    f = json.load(open(os.path.join(path_dir, "pmc_calibration_fetch.json")))
    w = json.load(open(os.path.join(path_dir, "pmc_calibration_write.json")))
    fr = [v for k, v in f.items() if k.split("/")[0] in ("rd16", "rd8", "lds16")]
    wr = [v for k, v in w.items() if k.split("/")[0] in ("wr16", "wr8")]
    return sum(fr) / len(fr), sum(wr) / len(wr)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--calib")]
    cdir = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--calib=")), "profiles/r6")
    f_ratio, w_ratio = _calib(cdir)
    fetch, fdur, calls = read_counter(args[0])
    write, _, _ = read_counter(args[1])
    stats = {}
    if len(args) > 2:
        with open(args[2]) as f:
            for r in csv.DictReader(f):
                stats[short(r["Name"])] = float(r["AverageNs"]) * 1e-3
    top = int(args[3]) if len(args) > 3 else 20
    rows = []
    for k in fetch:
        n = calls[k]
        us = stats.get(k, fdur[k] / n)
        fk, wk = fetch[k] / n / f_ratio, write.get(k, 0.0) / n / w_ratio
        rows.append((fk * n + wk * n, k, n, fk, wk, us, (fk + wk) * 1e3 / us / 1e6 if us > 0 else 0.0))
    rows.sort(reverse=True)
    print("# bytes corrected by the calibration ratios in %s: FETCH reported/true %.3f, WRITE %.3f" % (
        cdir, f_ratio, w_ratio))
    print("%-60s %6s %12s %12s %8s %7s %6s" % ("kernel", "calls", "read KB", "write KB", "us/call", "TB/s", "%peak"))
    for _, k, n, fk, wk, us, tbs in rows[:top]:
        print("%-60s %6d %12.1f %12.1f %8.2f %7.2f %5.0f%%" % (k[:60], n, fk, wk, us, tbs, 100 * tbs / 8.0))


if __name__ == "__main__":
    main()
