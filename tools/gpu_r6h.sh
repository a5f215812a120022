#!/bin/bash
# Round 6 (h): forward A/B (tools/build_kbench_r6.sh), two alternating passes.
set -o pipefail
OUT=gpurun_out/r6h
mkdir -p "$OUT"
for rep in 1 2; do
  for v in c2_base c2_srec c2_sf1 c2_sf2; do timeout -k 10 60 tools/bin/$v 1024 20 >> "$OUT/ab.txt" 2>&1 || exit 1; done
  for v in h_base h_sf1 h_sf2; do timeout -k 10 60 tools/bin/$v 2048 5 >> "$OUT/ab.txt" 2>&1 || exit 2; done
  for v in c5_base c5_sf1 c5_sf2; do timeout -k 10 60 tools/bin/$v 2048 3 >> "$OUT/ab.txt" 2>&1 || exit 3; done
done
