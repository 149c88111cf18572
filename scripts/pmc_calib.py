#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration from a rocprofv3 --pmc pass over
scripts/micro/pmc_calib (kernels that move a known 1 GiB each, read once per
launch from a buffer 4x the Infinity Cache).

usage: pmc_calib.py <counter_collection.csv> [<calib stdout jsonl>]

Prints, per kernel and counter, the median reported KB per launch and the
ratio to the true byte count. scripts/pmc_table.py reads the ratio file this
writes (--out) instead of assuming a factor."""
import csv
import json
import statistics
import sys
from collections import defaultdict

TRUE_BYTES = 1 << 30


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--out=")]
    outp = next((a[6:] for a in sys.argv[1:] if a.startswith("--out=")), None)
    vals = defaultdict(list)
    with open(args[0]) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            c = r["Counter_Name"]
            if c in ("FETCH_SIZE", "WRITE_SIZE"):
                vals[(k, c)].append(float(r["Counter_Value"]))   # KB
    ratios = {}
    for (k, c), v in sorted(vals.items()):
        kb = statistics.median(v)
        ratio = kb * 1024 / TRUE_BYTES
        ratios["%s/%s" % (k, c)] = ratio
        print("%-8s %-10s launches %2d  median %12.0f KB  true %10.0f KB  reported/true %.3f" % (
            k, c, len(v), kb, TRUE_BYTES / 1024, ratio))
    if outp:
        with open(outp, "w") as f:
            json.dump(ratios, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
