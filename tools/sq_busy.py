#!/usr/bin/env python3
"""SQ busy fractions per kernel from one rocprofv3 --pmc pass (run_counter_collection.csv).

    python tools/sq_busy.py gpurun_out/r3f/pmc_c2 [name-substring ...]

SIMD-cycles = GRBM_GUI_ACTIVE / 8 * 1024 (GRBM summed over the 8 XCDs, 1024 SIMDs).
  valu_busy       = SQ_ACTIVE_INST_VALU * 4 / SIMD-cycles (rocprof's VALUBusy; quad-cycle units).  It sums the
                    active cycles of every wave, so co-resident waves whose VALU work overlaps (the transcendental
                    unit, multi-pass fp64) count twice: it can exceed 1 and is NOT a utilisation.
  valu_issue      = SQ_INSTS_VALU * 4 / SIMD-cycles: the VALU issue slots used (a wave64 VALU instruction takes
                    4 cycles of a 16-lane SIMD), bounded by 1 except for transcendentals co-issued with VALU.
  fp64_flop_frac  = 64 (ADD + MUL + TRANS + 2 FMA)_F64 / (32 * SIMD-cycles): fp64 VALU FLOPs against the VALU
                    peak of 32 FLOP / SIMD / cycle (16 lanes x FMA), <= 1 by construction; fp32_flop_frac alike.
  mfma_busy       = SQ_VALU_MFMA_BUSY_CYCLES / SIMD-cycles.
Counters are summed over the dispatches of each kernel in the pass.  Prints one JSON list.
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
        def flops(p):
            keys = [f"SQ_INSTS_VALU_{op}_{p}" for op in ("ADD", "MUL", "TRANS", "FMA")]
            if not any(k in c for k in keys):
                return None
            return 64 * (sum(c.get(k, 0.0) for k in keys[:3]) + 2 * c.get(keys[3], 0.0)) / (32 * simd) if simd else None

        out.append({
            "kernel": name,
            "dispatches": n,
            "valu_busy": c.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / simd if simd and "SQ_ACTIVE_INST_VALU" in c else None,
            "valu_issue": c.get("SQ_INSTS_VALU", 0.0) * 4 / simd if simd and "SQ_INSTS_VALU" in c else None,
            "fp64_flop_frac": flops("F64"),
            "fp32_flop_frac": flops("F32"),
            "mfma_busy": c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / simd if simd and "SQ_VALU_MFMA_BUSY_CYCLES" in c else None,
            "valu_insts_per_dispatch": c.get("SQ_INSTS_VALU", 0.0) / n,
            "counters": dict(c),
        })
    out.sort(key=lambda r: -r["counters"].get("GRBM_GUI_ACTIVE", 0.0))
    return out


if __name__ == "__main__":
    print(json.dumps(summarize(sys.argv[1], tuple(sys.argv[2:])), indent=1))
