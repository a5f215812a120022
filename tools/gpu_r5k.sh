#!/bin/bash
# round 5: gradient suites at GTOL 1e-5, wide-channel parity after the MF K-quarter change, W46/W126 rows,
# the packed-FMA micro-benchmark and the gradient benchmark rows
set -e
mkdir -p gpurun_out/r5k
timeout -k 10 60 ./tools/bin/ubench_pk > gpurun_out/r5k/ubench_pk.jsonl 2>&1
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_wide_gpu.py > gpurun_out/r5k/wide.log 2>&1 || true
timeout -k 10 300 python -u tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 1 > gpurun_out/r5k/rows.jsonl 2> gpurun_out/r5k/rows.err
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_ho_grad_gpu.py tests/test_grad_gpu.py tests/test_long_grad_gpu.py > gpurun_out/r5k/grad.log 2>&1 || true
timeout -k 10 300 python -u tools/diag_ho_grad.py --quick --lengths 100,300,500 --out gpurun_out/r5k/diag.jsonl > gpurun_out/r5k/diag.log 2>&1
timeout -k 10 400 python -u tools/bench_grad.py --only gram,pde_gram,svgp126,svgp46,vosf_kdiag > gpurun_out/r5k/grad_bench.jsonl 2> gpurun_out/r5k/grad_bench.err
