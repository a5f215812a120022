#!/bin/bash
# the folded-weight normalised higher-order gradient (fp64 emission sides summed before rounding): A/B of the
# column-sum checkpoints and the fp64 emission, then the higher-order gradient tests
set -e
mkdir -p gpurun_out/r5f
for ck in 1 0; do for acc in 1 0; do
  GPSIG_HO_CKPT=$ck GPSIG_HO_ACC64=$acc timeout -k 10 200 python -u tools/diag_ho_grad.py --quick --lengths 100,500 \
    --out gpurun_out/r5f/ck${ck}_acc${acc}.jsonl > gpurun_out/r5f/ck${ck}_acc${acc}.log 2>&1
done; done
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_ho_grad_gpu.py > gpurun_out/r5f/hograd.log 2>&1
timeout -k 10 200 python -u tools/bench_pcie.py > gpurun_out/r5f/pcie.json 2> gpurun_out/r5f/pcie.err
