#!/bin/bash
# Round 6 (l): the kept split-f16 wide Gram (2 parts, per-row A scales): tests, W46 / W126 rows with a trace,
# one SQ counter pass over the two rows.
set -o pipefail
OUT=gpurun_out/r6l
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_wide_gpu.py tests/test_training_gpu.py tests/test_gram_gpu.py tests/test_long_gpu.py > "$OUT/tests.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.2 > "$OUT/rows.jsonl" 2> "$OUT/rows.err" || exit 2
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d "$OUT/sq" -o run --output-format csv -- \
  python3 tools/bench_rows.py --rows W46,W126 --reps 1 --cpu-seconds 0.2 > "$OUT/sq.log" 2>&1 || exit 3
timeout -k 10 300 python3 tools/diag_mf_precision.py > "$OUT/prec.jsonl" 2> "$OUT/prec.err" || exit 4
exit 0
