#!/bin/bash
# round 5, late: the whole GPU suite, smoke() and the default bench line on the current tree
set -o pipefail
OUT=gpurun_out/r5t
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> $OUT/gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
