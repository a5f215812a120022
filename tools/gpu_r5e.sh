#!/bin/bash
# A/B of the higher-order VJP's checkpoints and fp64 emission on the normalised order-5 gradient
set -e
mkdir -p gpurun_out/r5e
for ck in 1 0; do for acc in 1 0; do
  GPSIG_HO_CKPT=$ck GPSIG_HO_ACC64=$acc timeout -k 10 200 python -u tools/diag_ho_grad.py --quick --lengths 100,500 \
    --out gpurun_out/r5e/ck${ck}_acc${acc}.jsonl > gpurun_out/r5e/ck${ck}_acc${acc}.log 2>&1
done; done
