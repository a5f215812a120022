#!/usr/bin/env python3
"""Summarise the rocprofv3 passes of profiles/run_profile.sh into committed files.

    python profiles/summarize.py gpurun_out/prof r1

writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats summary, as produced),
profiles/<tag>_gram_counters.json (per-launch counters of the Gram kernel, HBM bytes with the gfx950
FETCH_SIZE correction of MI355X_MICROARCH.md 'HBM': bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024).
The Gram kernel is sig_fo_kernel with DIAGK = SAVE = false (the diagonal pass and the training
variant that saves the VJP state have their own symbols).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
here = os.path.dirname(os.path.abspath(__file__))


def is_gram(name):
    # sig_fo_kernel<DP, W, LP, M, SEED, DIAGK = false, SAVE = false, MF = false>
    # (a 9th argument, SPLIT = 0, follows MF in builds with the split diagnostic)
    return "sig_fo_kernel" in name and ("false, false, false>" in name or "false, false, false, 0>" in name
                                        or "Lb0ELb0ELb0E" in name)


def one(pattern):
    files = glob.glob(os.path.join(src, pattern), recursive=True)
    if not files:
        raise SystemExit(f"missing {pattern} under {src}")
    return files[0]


stats = one("trace/**/run_kernel_stats.csv")
shutil.copy(stats, os.path.join(here, f"{tag}_kernel_stats.csv"))
gram_stats = [r for r in csv.DictReader(open(stats)) if is_gram(r["Name"])]

per = defaultdict(list)
for sub in ("fetch", "write", "sq"):
    f = one(f"{sub}/**/run_counter_collection.csv")
    for r in csv.DictReader(open(f)):
        if is_gram(r["Kernel_Name"]):
            per[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in per.items()}
out = {
    "kernel": gram_stats[0]["Name"] if gram_stats else None,
    "launches_in_stats": int(gram_stats[0]["Calls"]) if gram_stats else None,
    "avg_duration_ms": float(gram_stats[0]["AverageNs"]) / 1e6 if gram_stats else None,
    "counters_per_launch": avg,
    "hbm_bytes_per_launch": (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024 if "FETCH_SIZE" in avg else None,
    "note": "FETCH_SIZE/WRITE_SIZE in KiB; FETCH doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B reads at 64 B)",
}
if "GRBM_GUI_ACTIVE" in avg and gram_stats:
    cycles = avg["GRBM_GUI_ACTIVE"] / 8  # summed over the 8 XCDs: shader cycles of the launch
    out["effective_clock_ghz"] = cycles / (out["avg_duration_ms"] * 1e6)
    simd_cycles = cycles * 1024  # 256 CUs x 4 SIMDs
    if "SQ_ACTIVE_INST_VALU" in avg:
        # measured busy counter (quad-cycles, MI355X_MICROARCH.md PMC units): fraction of the SIMDs'
        # cycles with a VALU instruction executing
        out["valu_busy"] = avg["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        out["mfma_busy"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
    if "SQ_WAVE_CYCLES" in avg:
        for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
            if k in avg:
                out[k.lower().replace("sq_", "") + "_per_wave_cycle"] = avg[k] / avg["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in avg:
        out["valu_insts_x4_over_simd_cycles"] = avg["SQ_INSTS_VALU"] * 4 / simd_cycles
json.dump(out, open(os.path.join(here, f"{tag}_gram_counters.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
