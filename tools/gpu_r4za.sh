#!/bin/bash
# Round-4: Kuf forward corner cells from additively carried exponents (|z0 - x|^2, <z0 - x, dz>) between
# exact passes: wide / training suites (corner-regime parity included), then the Kuf timing in both regimes
# against the previous commit (gpsig_amd/_ab/libgpsig_old.so).
OUT=${1:-gpurun_out/r4za}
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 900 $T tests/test_wide_gpu.py tests/test_training_gpu.py tests/test_grad_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
GPSIG_AMD_LIB=gpsig_amd/_ab/libgpsig_old.so timeout -k 10 300 python3 tools/bench_kuf_corner.py > "$OUT/kuf_old.jsonl" 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_kuf_corner.py > "$OUT/kuf_new.jsonl" 2>&1 || exit $?
grep -h "^{" "$OUT"/kuf_old.jsonl "$OUT"/kuf_new.jsonl
