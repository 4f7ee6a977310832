"""Summarise a rocprofv3 kernel trace (sqlite .db, or a kernel_stats.csv) per kernel:
calls, total ms, ms per step, average us; optionally the per-grid averages of one kernel.
Usage: prof_summary.py <db|csv> [steps] [kernel-name]"""

import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*$", "", name) if "<" not in name else name.split("(")[0]
    return name[:110]


def load(path):
    agg = defaultdict(lambda: [0, 0.0])
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur in c.execute("select name, (end - start) from kernels"):
            a = agg[short(name)]
            a[0] += 1
            a[1] += dur / 1e3
    else:
        for r in csv.DictReader(open(path)):
            a = agg[short(r["Name"])]
            a[0] += int(r["Calls"])
            a[1] += float(r["TotalDurationNs"]) / 1e3
    return agg


def main():
    agg = load(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':110s} {'calls':>7s} {'ms/step':>8s} {'avg_us':>8s} {'%':>6s}")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:110s} {n:7d} {us / 1e3 / steps:8.3f} {us / n:8.1f} {100 * us / tot:6.2f}")
    print(f"total GPU ms/step {tot / 1e3 / steps:.3f}")
    if len(sys.argv) > 3 and sys.argv[1].endswith(".db"):
        print(f"\nper-grid launches of {sys.argv[3]} (grid = workgroups x threads, as rocprof reports):")
        for gx, gy, gz, n, us in grid_breakdown(sys.argv[1], sys.argv[3]):
            print(f"  grid ({gx},{gy},{gz}) launches {n:6d} avg_us {us:8.2f}")


def grid_breakdown(path, kernel):
    """Per-launch-grid average duration of one kernel symbol (sqlite trace)."""
    c = sqlite3.connect(path)
    q = ("select grid_x, grid_y, grid_z, count(*), avg(end - start) from kernels "
         "where instr(name, ?) > 0 group by grid_x, grid_y, grid_z order by count(*) desc")
    return [(gx, gy, gz, n, us / 1e3) for gx, gy, gz, n, us in c.execute(q, (kernel,))]


if __name__ == "__main__":
    main()
