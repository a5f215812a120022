#!/bin/bash
# PDE adjoint A/B: parity of the PDE gradient tests, then the training-step timings with a trace
set -o pipefail
OUT=gpurun_out/r5q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pde_grad.py tests/test_pde_wide_gpu.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/grad" -o run --output-format csv -- python3 tools/bench_grad.py --reps 3 --only pde,pde_gram > "$OUT/grad_prof.log" 2>&1 || exit 2
timeout -k 10 300 python3 tools/bench_grad.py --reps 5 --only pde,pde_gram > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 3
