#!/bin/bash
set -e
mkdir -p gpurun_out/r5h
timeout -k 10 200 python -u tools/diag_ho_grad.py --quick --lengths 100,300,500 --out gpurun_out/r5h/diag.jsonl > gpurun_out/r5h/diag.log 2>&1
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_grad_gpu.py -k "far or corner" > gpurun_out/r5h/far.log 2>&1
