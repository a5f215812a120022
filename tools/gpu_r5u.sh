#!/bin/bash
# split higher-order VJP without slab barriers: parity + VOSF Kdiag timing with trace
set -o pipefail
OUT=gpurun_out/r5u
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ho_grad_gpu.py > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/grad" -o run --output-format csv -- python3 tools/bench_grad.py --reps 3 --only vosf_kdiag > "$OUT/grad_prof.log" 2>&1 || exit 2
timeout -k 10 300 python3 tools/bench_grad.py --reps 5 --only vosf_kdiag > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 3
