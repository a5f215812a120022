#!/bin/bash
# Counters of the VOSF Kff-diagonal training step (tools/bench_grad.py --only vosf_kdiag): the split higher-order
# forward and VJP.  One rocprofv3 --pmc pass per counter group.
set -o pipefail
OUT=${1:-gpurun_out/pmc_vosf}
mkdir -p $OUT
export TMPDIR=/tmp
RUN="python3 tools/bench_grad.py --reps 2 --only vosf_kdiag"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/a -o run --output-format csv -- $RUN > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -d $OUT/b -o run --output-format csv -- $RUN > $OUT/b.log 2>&1 || exit 2
python3 tools/sq_busy.py $OUT/a sig_ho > $OUT/a.json && python3 tools/sq_busy.py $OUT/b sig_ho > $OUT/b.json
