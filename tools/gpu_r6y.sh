#!/bin/bash
# Round 6 (y): anchor period 64 (default) against 128 at L = 128 (tools/kbench.hip), C5 and H.
set -o pipefail
OUT=gpurun_out/r6y
mkdir -p "$OUT"
for rep in 1 2; do
  for v in c5_w8lp16 c5_anch128 h_w8lp16 h_anch128; do timeout -k 10 120 tools/bin/$v 2048 5 >> "$OUT/ab.txt" 2>&1 || exit 1; done
done
