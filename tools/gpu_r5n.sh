#!/bin/bash
# round 5: gradient suites after the split-kernel last-point fix, the order-1 fold and the Kuf VJP |q| >= 2 rule;
# the split higher-order forward
set -e
mkdir -p gpurun_out/r5n
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_ho_grad_gpu.py tests/test_grad_gpu.py tests/test_long_grad_gpu.py tests/test_training_gpu.py tests/test_long_gpu.py > gpurun_out/r5n/grad.log 2>&1 || true
timeout -k 10 300 python -u tools/diag_ho_grad.py --quick --lengths 100,300,500 --out gpurun_out/r5n/diag.jsonl > gpurun_out/r5n/diag.log 2>&1
timeout -k 10 600 python -u tools/bench_grad.py --only gram,pde_gram,svgp126,svgp46,vosf_kdiag > gpurun_out/r5n/grad_bench.jsonl 2> gpurun_out/r5n/grad_bench.err
