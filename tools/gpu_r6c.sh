#!/bin/bash
# Round 6 (c): Gram-VJP A/B harness (tools/kbench_vjp.hip) -- the round-5 kernel vs the packed kernel -- and the
# SQ counters of the packed kernel with saved state.
set -o pipefail
OUT=gpurun_out/r6c
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in v_r5_st v_pk4_st v_pk4_st_wpe1 v_r5 v_pk4; do
  timeout -k 10 120 tools/bin/$v 1024 5 >> "$OUT/ab.txt" 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_pk4" -o run --output-format csv -- tools/bin/v_pk4_st 1024 2 > "$OUT/pmc_pk4.log" 2>&1 || exit 2
python3 tools/sq_busy.py "$OUT/pmc_pk4" > "$OUT/pmc_pk4.json" || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmc_r5" -o run --output-format csv -- tools/bin/v_r5_st 1024 2 > "$OUT/pmc_r5.log" 2>&1 || exit 4
python3 tools/sq_busy.py "$OUT/pmc_r5" > "$OUT/pmc_r5.json" || exit 5
