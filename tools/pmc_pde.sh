#!/bin/bash
# Counters of the PDE training step's adjoint launches (tools/bench_grad.py --only pde_gram): one rocprofv3
# --pmc pass per counter group (never with traces; FETCH_SIZE and WRITE_SIZE in passes of their own).
#   tools/pmc_pde.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/pmc_pde}
mkdir -p $OUT
export TMPDIR=/tmp
RUN="python3 tools/bench_grad.py --reps 2 --only pde_gram"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE -d $OUT/a -o run --output-format csv -- $RUN > $OUT/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 GRBM_GUI_ACTIVE -d $OUT/b -o run --output-format csv -- $RUN > $OUT/b.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $RUN > $OUT/fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $RUN > $OUT/write.log 2>&1 || exit 4
python3 tools/sq_busy.py $OUT/a pde_adj > $OUT/a.json && python3 tools/sq_busy.py $OUT/b pde_adj > $OUT/b.json
