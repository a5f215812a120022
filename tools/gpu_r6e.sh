#!/bin/bash
# Round 6 (e): segmented-scan radix A/B at C2 (tools/build_kbench_seg.sh), forward and VJP.
set -o pipefail
OUT=gpurun_out/r6e
mkdir -p "$OUT"
for rep in 1 2; do
  for v in c2f_r2 c2f_r4; do timeout -k 10 120 tools/bin/$v 1024 20 >> "$OUT/ab.txt" 2>&1 || exit 1; done
  for v in c2b_r2 c2b_r4; do timeout -k 10 120 tools/bin/$v 1024 5 >> "$OUT/ab.txt" 2>&1 || exit 2; done
done
