#!/bin/bash
# SQ / LDS counters of the Gram VJP launches of tools/prof_gram_vjp.py (one rocprofv3 --pmc pass each).
#   tools/pmc_vjp.sh <outdir>
OUT=${1:-gpurun_out/pmc_vjp}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 5 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/a -o run --output-format csv -- python3 tools/prof_gram_vjp.py > $OUT/a.log 2>&1 || exit 1
timeout -k 5 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $OUT/b -o run --output-format csv -- python3 tools/prof_gram_vjp.py > $OUT/b.log 2>&1 || exit 2
