#!/bin/bash
# Round 6 (u): headline profile passes and the C2 / C5 SQ pass on the final kernels (anchor period 64).
set -o pipefail
OUT=gpurun_out/r6u
mkdir -p "$OUT"
export TMPDIR=/tmp
bash profiles/run_profile.sh "$OUT/prof" || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d "$OUT/sq_rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows C2,C5 --reps 1 --cpu-seconds 0.2 > "$OUT/sq_rows.log" 2>&1 || exit 2
exit 0
