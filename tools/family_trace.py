"""Per-instance average duration of the roofline kernel family from a rocprofv3 kernel trace
of `bench.py --roofline-only N --roofline-case family` (one layer's set of family launches,
N times, nothing else on the GEMM kernels): dispatch k of every set is the same instance,
so averaging by position gives each instance's mean duration, to set beside the bench
line's live HIP-event numbers (roofline.instances[*].avg_launch_us).
    python tools/family_trace.py <run_results.db> <meta.json>"""

import json
import sqlite3
import sys


def main(db, metaf):
    meta = json.loads(open(metaf).read().strip().splitlines()[-1])
    per, n = meta["dispatches_per_launch"], meta["launches"]
    c = sqlite3.connect(db)
    match = meta.get("match") or [meta["kernel"]]  # a composite family lists its kernel names
    rows = [(nm, e - s) for nm, s, e in c.execute("select name, start, end from kernels order by start")
            if any(k in nm for k in match)]
    assert len(rows) == per * n, (len(rows), per, n)
    pos = [[] for _ in range(per)]
    for i, (nm, d) in enumerate(rows):
        pos[i % per].append(d)
    names = [rows[i][0].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "") for i in range(per)]
    out = {"sets": n, "per_set_us": sum(sum(p) for p in pos) / n / 1e3,
           "dispatch_avg_us": [round(sum(p) / len(p) / 1e3, 2) for p in pos], "kernels": names}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
