#!/bin/bash
# Round 6 (q): end-of-round evidence on the final kernels: the headline profile passes (trace, FETCH, WRITE,
# SQ), the C2 / C5 rows with a trace and an SQ pass, the gradient benchmark with a trace.
set -o pipefail
OUT=gpurun_out/r6q
mkdir -p "$OUT"
export TMPDIR=/tmp
bash profiles/run_profile.sh "$OUT/prof" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows C2,C5 --reps 5 --cpu-seconds 0.2 > "$OUT/rows.jsonl" 2> "$OUT/rows.err" || exit 2
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d "$OUT/sq_rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows C2,C5 --reps 1 --cpu-seconds 0.2 > "$OUT/sq_rows.log" 2>&1 || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/grad" -o run --output-format csv -- \
  python3 tools/bench_grad.py > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 4
exit 0
