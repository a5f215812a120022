#!/bin/bash
# Round-4: the Kuf forward's corner differences from the exact pass and the step's seeds (no second pass over
# the channels): the corner-regime test with the previous kernel (gpsig_amd/_ab/libgpsig_old.so) and the new
# one, the wide / training suites, the SVGP step timing.
OUT=${1:-gpurun_out/r4y}
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
GPSIG_AMD_LIB=gpsig_amd/_ab/libgpsig_old.so timeout -k 10 300 $T tests/test_wide_gpu.py -k corner > "$OUT/corner_old.log" 2>&1
r=$?; tail -1 "$OUT/corner_old.log"; [ $r -le 1 ] || exit $r
timeout -k 10 900 $T tests/test_wide_gpu.py tests/test_training_gpu.py tests/test_grad_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for D in 46 126; do
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
grep -h "^{" "$OUT"/svgp*.jsonl
