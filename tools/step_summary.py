"""Steady-state per-step kernel summary of a rocprofv3 kernel trace of bench.py (graphed
step): the dispatches between the optimizer kernels (adam_kernel) of the last N steps.
Reports launches per step, summed kernel time (busy) and wall time per step, then per
kernel name: launches/step, us/step, us/launch.
    python tools/step_summary.py <run_results.db> [N=5]"""

import collections
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    opt = [i for i, r in enumerate(rows) if "adam_kernel" in r[0]]
    assert len(opt) > n, "fewer optimizer steps than requested"
    seg = rows[opt[-n - 1] + 1:opt[-1] + 1]
    busy = sum(e - s for _, s, e in seg) / n / 1e6
    wall = (seg[-1][2] - seg[0][1]) / n / 1e6
    print(f"steady state over the last {n} steps: {len(seg) / n:.0f} launches/step, "
          f"busy {busy:.3f} ms/step, wall {wall:.3f} ms/step")
    tm, cnt = collections.Counter(), collections.Counter()
    for name, s, e in seg:
        k = name.replace("(anonymous namespace)::", "").replace("void ", "")
        k = re.sub(r"\(.*", "", k)
        tm[k] += e - s
        cnt[k] += 1
    print(f"{'kernel':100s} {'per step':>9s} {'us/step':>9s} {'us/launch':>9s}")
    for k, v in tm.most_common():
        print(f"{k[:100]:100s} {cnt[k] / n:9.1f} {v / n / 1e3:9.1f} {v / cnt[k] / 1e3:9.1f}")


if __name__ == "__main__":
    main()
