"""Summarise a rocprofv3 kernel trace (sqlite .db, or a kernel_stats.csv) per kernel:
calls, total ms, ms per step, average us.  Usage: prof_summary.py <db|csv> [steps]"""

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


if __name__ == "__main__":
    agg = load(sys.argv[1])
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':110s} {'calls':>7s} {'ms/step':>8s} {'avg_us':>8s} {'%':>6s}")
    for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:110s} {n:7d} {us / 1e3 / steps:8.3f} {us / n:8.1f} {100 * us / tot:6.2f}")
    print(f"total GPU ms/step {tot / 1e3 / steps:.3f}")
