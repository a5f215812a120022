#!/bin/bash
# Round 6 (t): anchor period 64 (GPSIG_PK_ANCHOR): the GPU suite, smoke and bench, C2 / C5 at steady state, the
# wide rows and the wide-path precision diagnostic.
set -o pipefail
OUT=gpurun_out/r6t
mkdir -p "$OUT"
export TMPDIR=/tmp
bash tools/gpu_suite.sh "$OUT/suite" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows C2,C5,W46,W126 --reps 30 --cpu-seconds 0.2 > "$OUT/rows.jsonl" 2> "$OUT/rows.err" || exit 2
timeout -k 10 300 python3 tools/diag_mf_precision.py > "$OUT/prec.jsonl" 2> "$OUT/prec.err" || exit 3
timeout -k 10 400 python3 tools/bench_grad.py --only gram,vosf_kdiag > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 4
exit 0
