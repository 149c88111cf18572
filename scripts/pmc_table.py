#!/usr/bin/env python3
"""Per-kernel memory traffic table from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE: kilobytes moved between L2 and memory, i.e.
HBM / MALL traffic, not L2 hits; on gfx950 FETCH_SIZE counts half the bytes
of wide coalesced 16-B-per-lane streaming reads -- MI355X_MICROARCH.md, HBM --
so the "fetch x2" column doubles it as the upper estimate) plus the kernel-trace durations of a
separate non-counter run (counter passes serialise dispatches, so their own
timestamps overstate short kernels).

usage: pmc_table.py FETCH_counter_collection.csv WRITE_counter_collection.csv
                    [kernel_stats.csv] [top N]
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


def main():
    fetch, fdur, calls = read_counter(sys.argv[1])
    write, _, _ = read_counter(sys.argv[2])
    stats = {}
    if len(sys.argv) > 3:
        with open(sys.argv[3]) as f:
            for r in csv.DictReader(f):
                stats[short(r["Name"])] = float(r["AverageNs"]) * 1e-3
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    rows = []
    for k in fetch:
        n = calls[k]
        us = stats.get(k, fdur[k] / n)
        fk, wk = fetch[k] / n, write.get(k, 0.0) / n
        rows.append((fk * n + wk * n, k, n, fk, wk, us, (fk + wk) * 1e3 / us / 1e6 if us > 0 else 0.0))
    rows.sort(reverse=True)
    print("%-60s %6s %10s %10s %10s %8s %7s %7s %6s" % ("kernel", "calls", "fetch KB", "fetchx2 KB", "write KB",
                                                        "us/call", "TB/s", "x2 TB/s", "%peak"))
    for _, k, n, fk, wk, us, tbs in rows[:top]:
        tb2 = (2 * fk + wk) * 1e3 / us / 1e6 if us > 0 else 0.0
        print("%-60s %6d %10.1f %10.1f %10.1f %8.2f %7.2f %7.2f %5.0f%%" % (k[:60], n, fk, 2 * fk, wk, us, tbs, tb2,
                                                                        100 * tb2 / 8.0))


if __name__ == "__main__":
    main()
