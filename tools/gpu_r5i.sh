#!/bin/bash
set -e
mkdir -p gpurun_out/r5i
for ck in 1 0; do for acc in 1 0; do
  GPSIG_HO_CKPT=$ck GPSIG_HO_ACC64=$acc timeout -k 10 200 python -u tools/diag_ho_grad.py --quick --lengths 500 \
    --out gpurun_out/r5i/ck${ck}_acc${acc}.jsonl > gpurun_out/r5i/ck${ck}_acc${acc}.log 2>&1
done; done
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_grad_gpu.py -k "far or corner" > gpurun_out/r5i/far.log 2>&1
