#!/bin/bash
# Round 6 (s): C2 and C5 rows at steady state (more launches per trace than the round's default 5 reps).
set -o pipefail
OUT=gpurun_out/r6s
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows C2,C5 --reps 30 --cpu-seconds 0.2 > "$OUT/rows.jsonl" 2> "$OUT/rows.err" || exit 1
exit 0
