#!/bin/bash
# VALU / MFMA busy counters of kbench variants (one rocprofv3 --pmc pass each).
#   tools/pmc_valu.sh <outdir> <variant>...
OUT=${1:-gpurun_out/pmc_valu}
shift
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 5 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $OUT/${v} -o run --output-format csv -- ./tools/bin/$v 2048 2 > $OUT/${v}.log 2>&1 || exit 1
done
