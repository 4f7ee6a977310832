"""Per-launch HBM traffic of the roofline kernel from two rocprofv3 PMC passes.

  rocprofv3 --pmc FETCH_SIZE -d <dir_f> -o run -- python3 bench.py --roofline-only 20
  rocprofv3 --pmc WRITE_SIZE -d <dir_w> -o run -- python3 bench.py --roofline-only 20
  python tools/pmc_traffic.py <dir_f>/run_results.db <dir_w>/run_results.db <meta.json> <out.json>

FETCH_SIZE / WRITE_SIZE are rocprof's derived kilobyte counters built on TCC_EA0_RDREQ /
_WRREQ (MI355X_MICROARCH.md §HBM); on gfx950 FETCH_SIZE reports half of the bytes of wide
coalesced streaming reads, so it is doubled here.  meta.json is the --roofline-only line."""

import json
import sqlite3
import statistics
import sys


def per_dispatch(db, counter, kernels):
    """Summed counter value per dispatch of any kernel whose name contains one of `kernels`
    (rocprofv3 counters_collection view), in dispatch order."""
    c = sqlite3.connect(db)
    q = ("select dispatch_id, kernel_name, sum(value) from counters_collection "
         "where counter_name = ? group by dispatch_id order by dispatch_id")
    return [v for _, name, v in c.execute(q, (counter,)) if any(k in name for k in kernels)]


if __name__ == "__main__":
    dbf, dbw, metaf, outf = sys.argv[1:5]
    meta = json.loads(open(metaf).read().strip().splitlines()[-1])
    names = meta.get("match") or [meta["kernel"]]  # a family lists its kernels' names
    f = per_dispatch(dbf, "FETCH_SIZE", names)
    w = per_dispatch(dbw, "WRITE_SIZE", names)
    assert f and w, "no dispatches of the roofline kernel in the PMC databases"
    per = meta.get("dispatches_per_launch", 1)
    if per > 1:  # a family: one "launch" = a layer's set of dispatches; total over the run / sets
        n = meta["launches"]
        assert len(f) == len(w) == n * per, (len(f), len(w), n, per)
        fk, wk = sum(f) / n, sum(w) / n
    else:
        fk, wk = statistics.median(f), statistics.median(w)
    out = {"kernel": meta["kernel"], "shape": meta["shape"], "build": meta.get("build"), "launches": [len(f), len(w)],
           "FETCH_SIZE_kB_per_launch": fk, "WRITE_SIZE_kB_per_launch": wk,
           "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
           "algorithmic_bytes_per_launch": meta["algorithmic_bytes_per_launch"],
           "note": "FETCH_SIZE doubled (gfx950 wide-read correction); kB = 1024 B"}
    json.dump(out, open(outf, "w"), indent=1)
    print(json.dumps(out))
