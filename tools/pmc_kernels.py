"""Per-kernel SQ counter summary of a rocprofv3 --pmc pass (counters_collection table of the
sqlite output): for each kernel name containing one of the given substrings, the mean per
dispatch of every collected counter, keyed by the library build (first 16 hex of its sha256).
    python tools/pmc_kernels.py <run_results.db> substr [substr ...]"""
import hashlib
import json
import os
import sqlite3
import sys
from collections import defaultdict


def main():
    db, subs = sys.argv[1], sys.argv[2:]
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection "
                     "group by dispatch_id, counter_name")
    acc = defaultdict(lambda: defaultdict(list))
    for _, name, cn, v in rows:
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if any(s in short for s in subs):
            acc[short][cn].append(v)
    out = {k: {cn: sum(v) / len(v) for cn, v in d.items()} | {"dispatches": max(len(v) for v in d.values())}
           for k, d in acc.items()}
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "liteasr_amd", "lib",
                       "libliteasr_hip.so")
    out["build"] = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
