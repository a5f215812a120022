#!/bin/bash
# Round 6 (f): gradient tests (closed-form scaling directions, RCCL world-1 data path), the gradient
# benchmark with a kernel trace, and one SQ counter pass over the Gram VJP.
set -o pipefail
OUT=gpurun_out/r6f
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_ho_grad_gpu.py tests/test_grad_gpu.py tests/test_rccl_gpu.py > "$OUT/tests.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 tools/bench_grad.py > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 2
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d "$OUT/sq" -o run \
  --output-format csv -- python3 tools/bench_grad.py --only gram --reps 2 > "$OUT/sq.log" 2>&1 || exit 3
exit 0
