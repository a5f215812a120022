#!/bin/bash
# Round 6 (g): baseline of the rows the verdict names (C2, C5, W46 traces; VOSF Kdiag backward) and the
# C2 forward harness on the same box.
set -o pipefail
OUT=gpurun_out/r6g
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 tools/bin/c2f_r2 1024 20 > "$OUT/kbench.txt" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows C2,C5,W46 --reps 3 --cpu-seconds 0.2 > "$OUT/rows.jsonl" 2> "$OUT/rows.err" || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/vosf" -o run --output-format csv -- \
  python3 tools/bench_grad.py --only vosf_kdiag > "$OUT/vosf.jsonl" 2> "$OUT/vosf.err" || exit 3
timeout -k 10 120 tools/bin/c2f_r2 1024 20 >> "$OUT/kbench.txt" 2>&1 || exit 4
exit 0
