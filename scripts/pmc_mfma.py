#!/usr/bin/env python3
"""Per-kernel MFMA utilisation and effective clock from one rocprofv3 --pmc
pass with SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (MI355X_MICROARCH.md:
MFMA busy cycles are summed over the SIMDs, GRBM_GUI_ACTIVE over the 8 XCDs):

  util  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  clock = GRBM_GUI_ACTIVE / 8 / kernel wall time  (reads high below ~0.3 ms)

usage: pmc_mfma.py counter_collection.csv [top N]"""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name
    for p in ("void ", "(anonymous namespace)::", "skr::"):
        n = n.replace(p, "")
    return n.split("(")[0].strip()[:64]


def main():
    busy, active, dur, calls = defaultdict(float), defaultdict(float), defaultdict(float), defaultdict(int)
    seen = set()
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            v = float(r["Counter_Value"])
            if r["Counter_Name"].startswith("SQ_VALU_MFMA_BUSY_CYCLES"):
                busy[k] += v
            elif r["Counter_Name"].startswith("GRBM_GUI_ACTIVE"):
                active[k] += v
            d = r["Dispatch_Id"]
            if d not in seen:
                seen.add(d)
                calls[k] += 1
                dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    rows = sorted(((active[k], k) for k in active), reverse=True)[:top]
    print("%-64s %6s %10s %9s %9s" % ("kernel", "calls", "us/call", "MFMA %", "GHz"))
    for _, k in rows:
        chip = active[k] / 8.0
        util = 100.0 * busy[k] / (chip * 1024) if chip > 0 else 0.0
        ghz = chip / dur[k] / 1e9 if dur[k] > 0 else 0.0
        print("%-64s %6d %10.2f %8.1f%% %9.2f" % (k, calls[k], 1e6 * dur[k] / calls[k], util, ghz))


if __name__ == "__main__":
    main()
