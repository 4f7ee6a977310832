"""Average PMC counter values per kernel from a rocprofv3 sqlite output.

    pmc_summary.py <db> [kernel-substring]
"""

import re
import sqlite3
import sys
from collections import defaultdict


def main():
    c = sqlite3.connect(sys.argv[1])
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    q = ("select kernel_name, dispatch_id, counter_name, value, duration, vgpr_count, accum_vgpr_count, "
         "sgpr_count, lds_block_size from counters_collection")
    per = defaultdict(lambda: defaultdict(list))
    meta = {}
    for name, disp, cn, val, dur, vg, ag, sg, lds in c.execute(q):
        if pat and pat not in name:
            continue
        k = re.sub(r"\(.*$", "", name)[:100]
        per[k][cn].append(val)
        per[k]["_dur_ns"].append(dur)
        meta[k] = (vg, ag, sg, lds)
    for k, d in per.items():
        print(k, "vgpr/agpr/sgpr/lds", meta[k])
        for cn, vals in sorted(d.items()):
            print(f"   {cn:28s} avg {sum(vals) / len(vals):16.1f}  n={len(vals)}")


if __name__ == "__main__":
    main()
