#!/bin/bash
# one-wave higher-order VJP with unfenced slab reads: parity + timings
set -o pipefail
OUT=gpurun_out/r5w
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ho_grad_gpu.py tests/test_grad_gpu.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_ho_vjp.py > $OUT/after.jsonl 2> $OUT/after.err || exit 2
