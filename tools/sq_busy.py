#!/usr/bin/env python3
"""SQ busy fractions per kernel from one rocprofv3 --pmc pass (run_counter_collection.csv).

    python tools/sq_busy.py gpurun_out/r3f/pmc_c2 [name-substring ...]

valu_busy = SQ_ACTIVE_INST_VALU * 4 / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)  (quad-cycle units, summed over
the 8 XCDs; MI355X_MICROARCH.md PMC table), mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 *
1024).  Counters are summed over the dispatches of each kernel in the pass.  Prints one JSON list.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarize(src, subs=()):
    files = glob.glob(os.path.join(src, "**", "run_counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no run_counter_collection.csv under {src}")
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if subs and not any(s in name for s in subs):
                continue
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[name].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    out = []
    for name, c in tot.items():
        simd = c.get("GRBM_GUI_ACTIVE", 0.0) / 8 * 1024
        n = max(len(disp[name]), 1)
        out.append({
            "kernel": name,
            "dispatches": n,
            "valu_busy": c.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / simd if simd else None,
            "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd if simd else None,
            "valu_insts_per_dispatch": c.get("SQ_INSTS_VALU", 0.0) / n,
            "counters": dict(c),
        })
    out.sort(key=lambda r: -r["counters"].get("GRBM_GUI_ACTIVE", 0.0))
    return out


if __name__ == "__main__":
    print(json.dumps(summarize(sys.argv[1], tuple(sys.argv[2:])), indent=1))
