#!/bin/bash
# PMC passes over kbench variants (each counter group in its own rocprofv3 run).
OUT=${OUT:-gpurun_out/pmc_kb}
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 5 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_BUSY_CYCLES -d $OUT/${v}_a -o run --output-format csv -- ./tools/bin/$v 2048 2 > $OUT/${v}_a.log 2>&1 || exit 1
  timeout -k 5 120 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LEVEL_WAVES SQ_ACTIVE_INST_MISC SQ_WAVES GRBM_GUI_ACTIVE -d $OUT/${v}_b -o run --output-format csv -- ./tools/bin/$v 2048 2 > $OUT/${v}_b.log 2>&1 || exit 2
done
