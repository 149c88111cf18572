#!/usr/bin/env python3
"""Per-kernel MFMA utilisation from one rocprofv3 --pmc pass with
SQ_VALU_MFMA_BUSY_CYCLES (busy cycles summed over the chip's 1,024 SIMDs).

  util = SQ_VALU_MFMA_BUSY_CYCLES / (kernel duration x 1024 SIMDs x 2.4 GHz)

The denominator uses the part's MAXIMUM clock (2.4 GHz, MI355X_MICROARCH.md
chip table) and the kernel-trace duration of the same dispatches, so the
figure is a LOWER bound on the fraction of available matrix cycles (the chip
holds a lower clock under MFMA load). No clock is derived from
GRBM_GUI_ACTIVE: that quotient reads high on dispatches shorter than about
0.3 ms (it gave 3-11 "GHz" for the recurrent per-step kernels in round 5);
it is printed only for dispatches of >= 0.3 ms, as a cross-check.

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
    rows = sorted(((busy[k], k) for k in busy), reverse=True)[:top]
    print("%-64s %6s %10s %13s %16s" % ("kernel", "calls", "us/call", "MFMA % (>=)", "GRBM GHz (>=0.3ms)"))
    for _, k in rows:
        avail = dur[k] * 1024 * 2.4e9
        util = 100.0 * busy[k] / avail if avail > 0 else 0.0
        per = dur[k] / calls[k]
        ghz = "%.2f" % (active[k] / 8.0 / dur[k] / 1e9) if (per >= 3e-4 and active.get(k)) else "-"
        print("%-64s %6d %10.2f %12.1f%% %16s" % (k, calls[k], 1e6 * per, util, ghz))


if __name__ == "__main__":
    main()
