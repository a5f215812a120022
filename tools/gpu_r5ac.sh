#!/bin/bash
# plain higher-order forward with interleaved scans: parity + secondary timings
set -o pipefail
OUT=gpurun_out/r5ac
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_long_gpu.py tests/test_ho_grad_gpu.py tests/test_gram_gpu.py tests/test_wide_gpu.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_secondary.py > $OUT/secondary.jsonl 2> $OUT/secondary.err || exit 2
timeout -k 10 300 python3 tools/bench_grad.py --reps 5 --only vosf_kdiag > $OUT/vosf.jsonl 2> $OUT/vosf.err || exit 3
