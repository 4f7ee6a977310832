"""Per-(kernel, grid) breakdown of a rocprofv3 kernel-trace db: calls/step, ms/step, avg us.
Usage: prof_grid.py <run_results.db> <steps> [top]"""
import collections
import sqlite3
import sys

db, steps = sys.argv[1], int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 50
c = sqlite3.connect(db)
agg = collections.defaultdict(lambda: [0, 0.0])
tot = 0.0
for name, gx, gy, gz, wx, dur in c.execute("select name, grid_x, grid_y, grid_z, workgroup_x, (end - start) from kernels"):
    a = agg[(name.replace("(anonymous namespace)::", "").split("(")[0][:72], f"{gx // max(wx, 1)},{gy},{gz}")]
    a[0] += 1
    a[1] += dur / 1e3
    tot += dur / 1e3
print(f"total {tot / steps / 1e3:.3f} ms/step over {steps} steps")
for (n, g), (cnt, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{n:74s} {g:>12s} {cnt / steps:6.1f} {t / steps / 1e3:7.3f}ms {t / cnt:8.1f}us")
