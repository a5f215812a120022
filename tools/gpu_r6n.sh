#!/bin/bash
# Round 6 (n): Gram VJP A/B of the cubic Ec + first-pair range check in the cell regeneration.
set -o pipefail
OUT=gpurun_out/r6n
mkdir -p "$OUT"
for rep in 1 2; do
  for v in v_r5_st v_r5_st_clo v_pk_l128 v_pk_l128_p0; do timeout -k 10 120 tools/bin/$v 1024 5 >> "$OUT/ab.txt" 2>&1 || exit 1; done
done
