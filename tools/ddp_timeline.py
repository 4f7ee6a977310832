"""Where the DDP bucket all-reduces land in the kernel timeline of a graphed step.

    python tools/ddp_timeline.py <run_results.db> [steps]

Reads a rocprofv3 kernel trace of ``bench.py --force-ddp`` (world-1 RCCL group, segmented
backward graphs) and, for the last step, prints each RCCL kernel with its start time
relative to the step's first kernel, and how many kernels and how much GPU time of the
step come after it (the backward still running behind the launched bucket)."""

import json
import sqlite3
import sys


def _is_comm(name):
    """RCCL kernels: the ring/tree collectives and, in a world-1 group, oneRankReduce."""
    n = name.lower()
    return "nccl" in n or "rccl" in n or "onerankreduce" in n


def main():
    db = sys.argv[1]
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    is_ar = [_is_comm(n) for n, _, _ in rows]
    # a step ends with the optimizer kernel; take the last adam launch as the step end
    ends = [i for i, (n, _, _) in enumerate(rows) if "adam_kernel" in n]
    if len(ends) < 2:
        raise SystemExit("need at least two steps in the trace")
    lo, hi = ends[-2] + 1, ends[-1]
    step = rows[lo:hi + 1]
    t0 = step[0][1]
    out = {"step_kernels": len(step), "step_span_us": round((step[-1][2] - t0) / 1e3, 1), "allreduce": []}
    for k, (n, s, e) in enumerate(step):
        if is_ar[lo + k]:
            after = step[k + 1:]
            busy_after = sum(x[2] - x[1] for x in after if not _is_comm(x[0]))
            out["allreduce"].append({"at_us": round((s - t0) / 1e3, 1), "dur_us": round((e - s) / 1e3, 1),
                                     "kernels_after": len(after), "gpu_us_after": round(busy_after / 1e3, 1),
                                     "name": n.split("(")[1 if n.startswith("void (") else 0][:60]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
