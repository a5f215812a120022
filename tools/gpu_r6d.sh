#!/bin/bash
# Round 6 (d): Gram-VJP A/B at L = 64 / 100 / 128 (tools/build_kbench_vjp.sh variants).
set -o pipefail
OUT=gpurun_out/r6d
mkdir -p "$OUT"
for v in v_r5_st v_pk4_st v_r5_l64 v_pk_l64 v_r5_l128 v_pk_l128; do
  timeout -k 10 120 tools/bin/$v 1024 5 >> "$OUT/ab.txt" 2>&1 || exit 1
done
