#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (``rocprofv3 --kernel-trace -d DIR``
writes ``DIR/*_results.db``): time per kernel name, divided by the number of
repetitions the traced program ran (per-step / per-call view).
usage: python scripts/prof_db.py <results.db> [reps] [top]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    reps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute("select %s, count(*), sum(end - start) from kernels group by %s order by 3 desc" % (name, name))
    rows = list(rows)
    tot = sum(r[2] for r in rows)
    print("total %.2f ms, per rep %.3f ms" % (tot / 1e6, tot / 1e6 / reps))
    for n, k, ns in rows[:top]:
        print("%9.3f ms/rep %7d calls %8.2f us avg  %s" % (ns / 1e6 / reps, k, ns / 1e3 / k, n[:100]))


if __name__ == "__main__":
    main()
