#!/bin/bash
# Round 6 (i): the split-f16 matrix-core wide Gram: wide / training tests, W46 / W126 rows with a trace.
set -o pipefail
OUT=gpurun_out/r6i
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_wide_gpu.py tests/test_training_gpu.py tests/test_gram_gpu.py > "$OUT/tests.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.2 > "$OUT/rows.jsonl" 2> "$OUT/rows.err" || exit 2
exit 0
