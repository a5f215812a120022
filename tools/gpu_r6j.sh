#!/bin/bash
# Round 6 (j): the split-f16 matrix-core Gram at narrow channel counts (GPSIG_FO_FIXED_MAX=0 sends every d to
# the wide kernels) against the fixed-d VALU kernels: H (bench.py), C2, C5.
set -o pipefail
OUT=gpurun_out/r6j
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/h_valu.json" 2> "$OUT/h_valu.err" || exit 1
GPSIG_FO_FIXED_MAX=0 timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > "$OUT/h_mf.json" 2> "$OUT/h_mf.err" || exit 2
GPSIG_FO_FIXED_MAX=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/mf" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows C2,C5 --reps 3 --cpu-seconds 0.2 > "$OUT/rows_mf.jsonl" 2> "$OUT/rows_mf.err" || exit 3
exit 0
