#!/bin/bash
# Evidence for the rows: kernel traces of C2 / C3 (kept LP=16, W=26 geometry) / C5 / W46 / W126 (matrix-core
# wide Gram) and SQ counter passes (VALU issue, fp64/fp32 FLOP fractions, MFMA busy), one --pmc pass each.
OUT=${1:-gpurun_out/r4h}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- python3 tools/bench_rows.py --rows C2,C3,C5,W46,W126 --reps 3 --cpu-seconds 1 --out "$OUT/rows.json" > "$OUT/rows.log" 2>&1 || exit $?
timeout -k 10 400 python3 tools/bench_rows.py --rows C2,C3,C5,W46,W126 --reps 5 --cpu-seconds 2 --out "$OUT/rows_noprof.json" > "$OUT/rows_noprof.log" 2>&1 || exit $?
F64="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
F32="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
pmc() {  # name rows counters...
  local name=$1 rows=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/pmc_$name" -o run --output-format csv -- python3 tools/bench_rows.py --rows $rows --reps 1 --cpu-seconds 0.2 > "$OUT/pmc_$name.log" 2>&1 || return 1
  python3 tools/sq_busy.py "$OUT/pmc_$name" > "$OUT/pmc_$name.json" || return 2
}
pmc c3_f64 C3 $F64 || exit 11
pmc c2_f32 C2 $F32 || exit 12
pmc c5_f32 C5 $F32 || exit 13
pmc w46_mf W46 $MF || exit 14
pmc w126_mf W126 $MF || exit 15
pmc w126_f32 W126 $F32 || exit 16
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4h/pmc_*.json")):
    for r in json.load(open(f))[:3]:
        print(f.split("/")[-1], r["kernel"][:60], r["dispatches"], {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items() if k in ("valu_busy", "valu_issue", "fp64_flop_frac", "fp32_flop_frac", "mfma_busy")})
PY
