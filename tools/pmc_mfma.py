"""MFMA utilisation from a rocprofv3 PMC pass (SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE).

  rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d D -o run \
      -- python3 bench.py --graph off --steps 3 --warmup 1 --no-cpu-baseline --no-roofline
  python tools/pmc_mfma.py D/run_counter_collection.csv [CONFIG]

Per dispatch: elapsed shader cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs,
MI355X_MICROARCH.md "DVFS give-back"); MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES /
(elapsed x 1024 SIMDs) (busy counts SIMD cycles, 32 per v_mfma_f32_32x32x16_bf16, ibid.
"s_memtime tick vs SQ PMC units").  Prints one JSON object: the whole run's
cycle-weighted utilisation and the top kernels by elapsed cycles.
"""

import csv
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4


def case_summary(path, meta_path):
    """MFMA utilisation over the dispatches of one roofline case (bench.py --roofline-only N
    --roofline-case C under the counter pass): kernels whose names contain one of meta["match"]."""
    meta = json.load(open(meta_path))
    busy = el = 0.0
    n = 0
    rows = defaultdict(lambda: defaultdict(float))
    name = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = r.get("Dispatch_Id") or r.get("Dispatch_ID") or r.get("Correlation_Id")
            name[d] = r.get("Kernel_Name", "?")
            rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
    for d, c in rows.items():
        if any(m in name[d] for m in meta["match"]) and "GRBM_GUI_ACTIVE" in c:
            busy += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            el += c["GRBM_GUI_ACTIVE"] / 8.0
            n += 1
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import build_key

    print(json.dumps({"build": build_key(), "kernel": meta["kernel"], "shape": meta["shape"], "dispatches": n,
                      "mfma_util": busy / (el * SIMDS) if el else None,
                      "note": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs) over the case's "
                              "dispatches (counter mode serialises dispatches)"}, indent=1))


def main(path, config="small"):
    rows = defaultdict(lambda: defaultdict(float))  # dispatch id -> counter -> value
    name = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            d = r.get("Dispatch_Id") or r.get("Dispatch_ID") or r.get("Correlation_Id")
            name[d] = r.get("Kernel_Name", "?")
            rows[d][r["Counter_Name"]] += float(r["Counter_Value"])
    per = defaultdict(lambda: [0, 0.0, 0.0])  # kernel -> launches, busy, elapsed
    for d, c in rows.items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or "GRBM_GUI_ACTIVE" not in c:
            continue
        k = name[d].replace("(anonymous namespace)::", "").split("(")[0][:90]
        per[k][0] += 1
        per[k][1] += c["SQ_VALU_MFMA_BUSY_CYCLES"]
        per[k][2] += c["GRBM_GUI_ACTIVE"] / 8.0
    busy = sum(v[1] for v in per.values())
    el = sum(v[2] for v in per.values())
    top = sorted(per.items(), key=lambda kv: -kv[1][2])[:15]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import build_key  # the library build the pass measured (bench.pmc_mfma matches on it)

    out = {
        "build": build_key(), "config": config,
        "dispatches": sum(v[0] for v in per.values()),
        "mfma_util_all_kernels": busy / (el * SIMDS) if el else None,
        "elapsed_cycles_sum": el,
        "top_kernels": [{"kernel": k, "launches": v[0], "elapsed_share": v[2] / el,
                         "mfma_util": v[1] / (v[2] * SIMDS) if v[2] else None} for k, v in top],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 3 and sys.argv[2] == "--case":
        case_summary(sys.argv[1], sys.argv[3])
    else:
        main(sys.argv[1], *(sys.argv[2:3]))
