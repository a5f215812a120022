#!/bin/bash
# Round 6 (x): forward geometry A/B at L = 128 (tools/kbench.hip): W = 8 x LP = 16 (the default) against
# W = 4 x LP = 32, for C5 (D = 8, M = 6) and H (D = 5, M = 5).
set -o pipefail
OUT=gpurun_out/r6x
mkdir -p "$OUT"
for rep in 1 2; do
  for v in c5_w8lp16 c5_w4lp32; do timeout -k 10 120 tools/bin/$v 2048 5 >> "$OUT/ab.txt" 2>&1 || exit 1; done
  for v in h_w8lp16 h_w4lp32; do timeout -k 10 120 tools/bin/$v 2048 5 >> "$OUT/ab.txt" 2>&1 || exit 2; done
done
