#!/bin/bash
# rocprofv3 passes for the headline bench (run on the GPU box from the repo root, via gpurun).
# Pass 1: kernel trace + stats.  Passes 2-4: PMC counters, each in its own run (--pmc never combined
# with sys/runtime/hip traces; FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
set -o pipefail
OUT=${1:-gpurun_out/prof}
ARGS=${2:-"--steps 2 --warmup 1 --no-cpu --no-check"}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS > $OUT/write.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 || exit 4
exit 0
