#!/bin/bash
# Round 6 (r): the PDE forward with an fp32 solution grid (tools/bin/lib_pde32.so, GPSIG_PDE_T=float) against the
# fp64 grid: C3 row (time, max-abs error vs the reference's own Cython-restated oracle) and the PDE tests.
set -o pipefail
OUT=gpurun_out/r6r
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_rows.py --rows C3 --reps 5 --cpu-seconds 0.2 > "$OUT/c3_f64.jsonl" 2> "$OUT/c3_f64.err" || exit 1
GPSIG_AMD_LIB=$PWD/tools/bin/lib_pde32.so timeout -k 10 300 python3 tools/bench_rows.py --rows C3 --reps 5 --cpu-seconds 0.2 > "$OUT/c3_f32.jsonl" 2> "$OUT/c3_f32.err" || exit 2
GPSIG_AMD_LIB=$PWD/tools/bin/lib_pde32.so timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_pde_gpu.py > "$OUT/pde32_tests.log" 2>&1
exit 0
