#!/usr/bin/env python3
"""Summarise rocprofv3 SQLite output (rocpd *_results.db) into small CSVs for profiles/.

    python tools/rocpd_summary.py stats  <db> [out.csv]   per-kernel calls / total / avg ns / %
    python tools/rocpd_summary.py pmc    <db> [out.csv]   per-kernel per-counter sum and mean per dispatch

FETCH_SIZE / WRITE_SIZE are reported as rocprofv3 gives them (KiB); the gfx950 correction
(MI355X_MICROARCH.md, HBM: FETCH_SIZE counts half the bytes of wide coalesced reads) is
applied by the reader, not here.
"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                     "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    out = [["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"]]
    for n, k, s, a, mn, mx in rows:
        out.append([n, k, int(s), round(a, 1), round(100.0 * s / total, 2), int(mn), int(mx)])
    return out


def pmc(db):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, count(*), sum(value), avg(value) from counters_collection "
                     "group by kernel_name, counter_name order by kernel_name, counter_name").fetchall()
    dur = dict(c.execute("select name, avg(duration) from kernels group by name").fetchall())
    out = [["Kernel", "Counter", "Dispatches", "Sum", "MeanPerDispatch", "AvgDurationNs"]]
    for kn, cn, k, s, a in rows:
        out.append([kn, cn, k, s, round(a, 3), round(dur.get(kn, 0.0), 1)])
    return out


def main():
    mode, db = sys.argv[1], sys.argv[2]
    rows = {"stats": stats, "pmc": pmc}[mode](db)
    f = open(sys.argv[3], "w", newline="") if len(sys.argv) > 3 else sys.stdout
    csv.writer(f).writerows(rows)


if __name__ == "__main__":
    main()
