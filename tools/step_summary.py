"""Steady-state per-step kernel summary of a rocprofv3 kernel trace of bench.py (graphed
step): the dispatches between the optimizer kernels (adam_kernel) of the last N steps.
Reports launches per step, summed kernel time (busy) and wall time per step, then per
kernel name: launches/step, us/step, us/launch.  --grid splits each kernel by its grid size
(workgroups x, y, z), which tells apart the GEMM shapes sharing one tile instance; --order
prints the last step's launches in order (name, grid, us) instead.
    python tools/step_summary.py <run_results.db> [N=5] [--grid] [--order]"""

import collections
import re
import sqlite3
import sys


def main():
    argv = [a for a in sys.argv[1:] if a not in ("--grid", "--order")]
    grid = "--grid" in sys.argv or "--order" in sys.argv
    db = argv[0]
    n = int(argv[1]) if len(argv) > 1 else 5
    c = sqlite3.connect(db)
    rows = [(f"{nm} [{gx // max(wx, 1)}x{gy // max(wy, 1)}x{gz // max(wz, 1)}]" if grid else nm, s, e)
            for nm, s, e, gx, gy, gz, wx, wy, wz in
            c.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, workgroup_z "
                      "from kernels order by start")]
    opt = [i for i, r in enumerate(rows) if "adam_kernel" in r[0]]
    assert len(opt) > n, "fewer optimizer steps than requested"
    seg = rows[opt[-n - 1] + 1:opt[-1] + 1]
    busy = sum(e - s for _, s, e in seg) / n / 1e6
    wall = (seg[-1][2] - seg[0][1]) / n / 1e6
    print(f"steady state over the last {n} steps: {len(seg) / n:.0f} launches/step, "
          f"busy {busy:.3f} ms/step, wall {wall:.3f} ms/step")
    if "--order" in sys.argv:
        last = rows[opt[-2] + 1:opt[-1] + 1]
        for i, (name, s_, e_) in enumerate(last):
            k = re.sub(r"\(.*\)", "", name.replace("(anonymous namespace)::", "").replace("void ", ""))
            print(f"{i:4d} {(e_ - s_) / 1e3:8.1f} {(s_ - last[0][1]) / 1e3:9.1f}  {k[:150]}")
        return
    tm, cnt = collections.Counter(), collections.Counter()
    for name, s, e in seg:
        k = name.replace("(anonymous namespace)::", "").replace("void ", "")
        k = re.sub(r"\(.*\)", "", k)
        tm[k] += e - s
        cnt[k] += 1
    print(f"{'kernel':110s} {'per step':>9s} {'us/step':>9s} {'us/launch':>9s}")
    for k, v in tm.most_common():
        print(f"{k[:110]:110s} {cnt[k] / n:9.1f} {v / n / 1e3:9.1f} {v / cnt[k] / 1e3:9.1f}")


if __name__ == "__main__":
    main()
