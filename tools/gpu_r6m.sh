#!/bin/bash
# Round 6 (m): forward A/B of the first-pair-only range check (tools/build_kbench_plo.sh), two passes.
set -o pipefail
OUT=gpurun_out/r6m
mkdir -p "$OUT"
for rep in 1 2; do
  for v in c2_base c2_plo; do timeout -k 10 60 tools/bin/$v 1024 20 >> "$OUT/ab.txt" 2>&1 || exit 1; done
  for v in h_base h_plo; do timeout -k 10 60 tools/bin/$v 2048 5 >> "$OUT/ab.txt" 2>&1 || exit 2; done
  for v in c5_base c5_plo; do timeout -k 10 60 tools/bin/$v 2048 3 >> "$OUT/ab.txt" 2>&1 || exit 3; done
done
