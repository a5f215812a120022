#!/bin/bash
# gradient suites at GTOL 1e-5 (round-4 verdict item 1) + the normalised higher-order diagnostics
set -e
mkdir -p gpurun_out/r5j
timeout -k 10 200 python -u tools/diag_ho_grad.py --lengths 100,300,500 --out gpurun_out/r5j/diag.jsonl > gpurun_out/r5j/diag.log 2>&1
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_ho_grad_gpu.py tests/test_grad_gpu.py tests/test_long_grad_gpu.py > gpurun_out/r5j/grad.log 2>&1 || true
timeout -k 10 60 ./tools/bin/ubench_pk > gpurun_out/r5j/ubench_pk.jsonl 2>&1
timeout -k 10 300 python -u tools/bench_grad.py --only gram,pde_gram,svgp126,svgp46,vosf_kdiag > gpurun_out/r5j/grad_bench.jsonl 2> gpurun_out/r5j/grad_bench.err
