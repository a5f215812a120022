#!/bin/bash
# Round-4: the DIAG tiles' anchor kernel with 8 anchor rows per thread (x_i as scalar loads): the wide and
# gradient suites that build the tiles, the SVGP step timing and its kernel trace.
OUT=${1:-gpurun_out/r4x}
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 900 $T tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_training_gpu.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for D in 46 126; do
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
grep -h "^{" "$OUT"/svgp*.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_svgp126" -o run --output-format csv -- python3 tools/bench_grad.py --only svgp126 --reps 3 > "$OUT/prof_svgp126.log" 2>&1 || exit $?
