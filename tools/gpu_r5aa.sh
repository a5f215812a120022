#!/bin/bash
# MF Gram: 8 waves (2 per SIMD, 256-VGPR cap) vs 4 waves per workgroup at W46 / W126
set -o pipefail
OUT=gpurun_out/r5aa
mkdir -p $OUT
timeout -k 10 300 python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.2 --out $OUT/nw8.json > $OUT/nw8.log 2>&1 || exit 1
GPSIG_MF_NW=4 timeout -k 10 300 python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.2 --out $OUT/nw4.json > $OUT/nw4.log 2>&1 || exit 2
