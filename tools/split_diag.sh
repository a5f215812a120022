#!/bin/bash
# The split design of SURVEY.md 8d as a diagnostic (bench.py --gram-path split): kernel trace of the
# producer / consumer launches and the consumer's HBM bytes (FETCH_SIZE, WRITE_SIZE passes).
#   tools/split_diag.sh <outdir>
OUT=${1:-gpurun_out/split}
ARGS="--gram-path split --steps 2 --warmup 1 --no-cpu --no-probe"
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS --no-check > $OUT/trace.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $ARGS --no-check > $OUT/fetch.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $ARGS --no-check > $OUT/write.log 2>&1 || exit 4
exit 0
