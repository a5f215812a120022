#!/bin/bash
# Kuf forward exact-value rule without the per-component underflow ballot: parity + C4/C4i rows with trace
set -o pipefail
OUT=gpurun_out/r5p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tensors_gpu.py tests/test_grad_gpu.py tests/test_wide_gpu.py -k "tens_vs_seq or kuf or far" > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- python3 tools/bench_rows.py --rows C4,C4i --reps 3 --cpu-seconds 0.5 --out "$OUT/rows_prof.json" > "$OUT/rows_prof.log" 2>&1 || exit 2
timeout -k 10 300 python3 tools/bench_rows.py --rows C4,C4i --reps 5 --cpu-seconds 1 --out "$OUT/rows.json" > "$OUT/rows.log" 2>&1 || exit 3
