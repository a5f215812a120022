#!/bin/bash
# PDE adjoint (front prefetch, batched dx reads) and signature features past the LDS
set -o pipefail
OUT=gpurun_out/r5r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pde_grad.py tests/test_pde_wide_gpu.py tests/test_signatures.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/grad" -o run --output-format csv -- python3 tools/bench_grad.py --reps 3 --only pde,pde_gram,sig > "$OUT/grad_prof.log" 2>&1 || exit 2
timeout -k 10 300 python3 tools/bench_grad.py --reps 5 --only pde,pde_gram,sig > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 3
