#!/bin/bash
# Kuf chunked seed tiles + the halved x-dot GEMM: wide / grad tests, SVGP timing; then the headline bench's
# rocprofv3 passes for round 4 (profiles/run_profile.sh).
OUT=${1:-gpurun_out/r4n}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_training_gpu.py tests/test_ho_grad_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
r=$?; tail -3 "$OUT/pytest.log"; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
for D in 46 126; do
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
cat "$OUT"/svgp*.jsonl | grep "^{"
bash profiles/run_profile.sh gpurun_out/prof_r4 || exit $?
