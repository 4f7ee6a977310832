"""Per-kernel, per-grid summary of a rocprofv3 kernel trace (run_results.db): calls per step,
average us, ms per step, scratch bytes.  Usage: trace_grid.py <db> [steps] [name-filter] [top]"""
import re
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 10.0
filt = sys.argv[3] if len(sys.argv) > 3 else ""
top = int(sys.argv[4]) if len(sys.argv) > 4 else 45
c = sqlite3.connect(db)
agg = defaultdict(lambda: [0, 0.0, 0])
for name, dur, gx, gy, gz, wx, scr in c.execute(
        "select name, duration, grid_x, grid_y, grid_z, workgroup_x, scratch_size from kernels"):
    n = re.sub(r"^void ", "", name.split("(")[0])
    n = re.sub(r"\(anonymous namespace\)::", "", n)[:72]
    if filt and filt not in n:
        continue
    a = agg[(n, gx // max(wx, 1), gy, gz)]
    a[0] += 1
    a[1] += dur / 1e3
    a[2] = scr
tot = sum(a[1] for a in agg.values())
print(f"total {tot / steps / 1e3:.3f} ms per step ({steps:g} steps)")
for k, a in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{k[0]:72s} {k[1]:5d}x{k[2]:5d}x{k[3]:3d} {a[0] / steps:6.1f}/st {a[1] / a[0]:8.1f} us "
          f"{a[1] / steps / 1e3:7.3f} ms/st scr {a[2]}")
