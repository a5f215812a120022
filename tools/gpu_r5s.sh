#!/bin/bash
# order-6 higher-order VJP; PDE + signature tests
set -o pipefail
OUT=gpurun_out/r5s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ho_grad_gpu.py tests/test_pde_grad.py tests/test_pde_wide_gpu.py tests/test_signatures.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/bench_grad.py --reps 5 --only pde,pde_gram,sig > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 3
