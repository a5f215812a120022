#!/bin/bash
# Round-4 A/B of the fp32 GEMM's row-major operand loads (lane per row -> 16 lanes along K per row):
# (then the 16-byte epilogue on the transposed accumulator and 16-byte k-major loads; then 16-byte
# row-major loads, A/B against the previous commit)
# tools/bench_gemm.py with the previous loads (gpsig_amd/_ab/libgpsig_old.so) and the new ones, the GEMM
# parity test, the wide / gradient suites that call the GEMM, then the SVGP step timing.
OUT=${1:-gpurun_out/r4t}
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
GPSIG_AMD_LIB=gpsig_amd/_ab/libgpsig_old.so timeout -k 10 300 python3 tools/bench_gemm.py > "$OUT/gemm_old.jsonl" 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_gemm.py > "$OUT/gemm_new.jsonl" 2>&1 || exit $?
cat "$OUT/gemm_old.jsonl" "$OUT/gemm_new.jsonl"
timeout -k 10 900 $T tests/test_gemm_gpu.py tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_pde_wide_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for D in 46 126; do
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
grep -h "^{" "$OUT"/svgp*.jsonl
