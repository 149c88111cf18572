#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_stats.csv: per-step ms by kernel."""
import csv, sys
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print("total %.2f ms, per step %.2f ms" % (tot / 1e6, tot / 1e6 / steps))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    print("%8.3f ms/step %6d calls %8.2f us avg  %s" % (float(r['TotalDurationNs']) / 1e6 / steps, int(r['Calls']),
                                                    float(r['AverageNs']) / 1e3, r['Name'][:90]))
