#!/bin/bash
# 8-wave split higher-order VJP past 509 points: parity, then the whole HO/grad suites
set -o pipefail
OUT=gpurun_out/r5y
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_ho_grad_gpu.py -k "past_512 or unsupported" > $OUT/tests_new.log 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ho_grad_gpu.py tests/test_grad_gpu.py tests/test_long_grad_gpu.py > $OUT/tests.log 2>&1 || exit 2
timeout -k 10 300 python3 tools/bench_ho_vjp.py > $OUT/ho_vjp.jsonl 2> $OUT/ho_vjp.err || exit 3
