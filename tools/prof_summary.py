#!/usr/bin/env python3
"""Summarise a rocprofv3 run (SQLite .db or kernel_stats.csv) into a text table.

usage: tools/prof_summary.py <results.db | kernel_stats.csv> [out.txt]
"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    # per-dispatch durations (ns) grouped by kernel name
    q = ("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
         "from kernels group by name order by sum(duration) desc")
    try:
        return [(r[0], r[1], r[2], r[3], r[4], r[5]) for r in c.execute(q)]
    except sqlite3.OperationalError:
        out = []
        for r in c.execute("select name,total_calls,total_duration,average from top_kernels"):
            out.append((r[0], r[1], r[2], r[3], None, None))
        return out


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                        float(r.get("MinNs", 0) or 0), float(r.get("MaxNs", 0) or 0)))
    return out


def main():
    src = sys.argv[1]
    rows = rows_from_db(src) if src.endswith(".db") else rows_from_csv(src)
    tot = sum(r[2] for r in rows) or 1
    lines = [f"# rocprofv3 --kernel-trace --stats summary of {src.split('/')[-1]}",
             f"{'kernel':40s} {'calls':>6s} {'total_ms':>10s} {'avg_ms':>10s} {'min_ms':>10s} {'max_ms':>10s} {'pct':>6s}"]
    for name, n, t, a, mn, mx in rows:
        f = lambda v: f"{v / 1e6:10.3f}" if v is not None else f"{'-':>10s}"
        lines.append(f"{name[:40]:40s} {n:6d} {f(t)} {f(a)} {f(mn)} {f(mx)} {100 * t / tot:6.2f}")
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
