"""Per-(kernel, grid) breakdown of a rocprofv3 sqlite kernel trace, plus GPU idle time.

    prof_shapes.py <trace.db> <steps> [top]

Prints the top (kernel, grid) pairs by total time per step, and the busy/idle split over
the trace span (idle = gaps between consecutive kernels: launch overhead / host-bound time).
"""

import re
import sqlite3
import sys
from collections import defaultdict


def short(name):
    return re.sub(r"\(.*$", "", name)[:90]


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, grid_x, grid_y, grid_z, start, end from kernels order by start"))
    agg = defaultdict(lambda: [0, 0.0])
    for name, gx, gy, gz, s, e in rows:
        a = agg[(short(name), gx, gy, gz)]
        a[0] += 1
        a[1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':90s} {'grid':>18s} {'n/step':>7s} {'ms/step':>8s} {'avg_us':>8s}")
    for (k, gx, gy, gz), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{k:90s} {f'{gx},{gy},{gz}':>18s} {n / steps:7.1f} {us / 1e3 / steps:8.3f} {us / n:8.1f}")
    print(f"total kernel ms/step {tot / 1e3 / steps:.3f}  launches/step {len(rows) / steps:.0f}")
    # idle gaps over the last 60 % of launches (past warm-up)
    n_last = int(len(rows) * 0.6)
    tail = rows[-n_last:]
    busy = sum(e - s for _, _, _, _, s, e in tail)
    span = tail[-1][5] - tail[0][4]
    gaps = []
    prev_end = tail[0][5]
    for _, _, _, _, s, e in tail[1:]:
        gaps.append(max(0, s - prev_end))
        prev_end = max(prev_end, e)
    gaps.sort()
    print(f"tail: {len(tail)} launches span {span / 1e6:.2f} ms busy {busy / 1e6:.2f} ms "
          f"idle {100 * (1 - busy / span):.1f}%  median gap {gaps[len(gaps) // 2] / 1e3:.2f} us "
          f"p90 gap {gaps[int(len(gaps) * 0.9)] / 1e3:.2f} us")


if __name__ == "__main__":
    main()
