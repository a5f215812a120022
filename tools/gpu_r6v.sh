#!/bin/bash
# Round 6 (v): PDE adjoint chunk-length A/B (GPSIG_PDE_HF 32 vs 64 corner floats per lane) plus its gradient tests.
set -o pipefail
OUT=gpurun_out/r6v
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 python3 tools/bench_grad.py --only pde_gram >> "$OUT/ab.txt" 2>&1 || exit 1
  GPSIG_AMD_LIB=$PWD/tools/bin/lib_pdeh64.so timeout -k 10 120 python3 tools/bench_grad.py --only pde_gram | sed 's/^/h64 /' >> "$OUT/ab.txt" 2>&1 || exit 2
done
GPSIG_AMD_LIB=$PWD/tools/bin/lib_pdeh64.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_pde_grad.py tests/test_pde_gpu.py -m gpu > "$OUT/tests_h64.txt" 2>&1 || exit 3
exit 0
