#!/bin/bash
set -o pipefail
OUT=gpurun_out/r5ad
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_signatures.py tests/test_ho_grad_gpu.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_grad.py --reps 5 --only sig > $OUT/sig.jsonl 2> $OUT/sig.err || exit 2
