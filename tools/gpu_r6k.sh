#!/bin/bash
# Round 6 (k): split-f16 wide Gram with per-row A scales: precision vs the fp64 oracle (and the fp32 channel
# loop), wide / training / Gram tests, W46 / W126 rows with 3 and 2 operand parts.
set -o pipefail
OUT=gpurun_out/r6k
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag_mf_precision.py > "$OUT/prec.jsonl" 2> "$OUT/prec.err" || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_wide_gpu.py tests/test_training_gpu.py tests/test_gram_gpu.py tests/test_long_gpu.py > "$OUT/tests.log" 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.2 > "$OUT/rows.jsonl" 2> "$OUT/rows.err" || exit 3
GPSIG_MF_PARTS=2 timeout -k 10 300 python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.2 > "$OUT/rows_np2.jsonl" 2> "$OUT/rows_np2.err" || exit 4
GPSIG_MF_PARTS=2 timeout -k 10 300 python3 tools/diag_mf_precision.py > "$OUT/prec_np2.jsonl" 2> "$OUT/prec_np2.err" || exit 5
exit 0
