#!/bin/bash
# round 5 final: the whole GPU suite, smoke(), the bench line, and the gradient benchmark with its trace
set -o pipefail
OUT=gpurun_out/r5x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/gpu_suite.log 2>&1
rc=$?
echo "suite rc=$rc" >> $OUT/gpu_suite.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 3
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/grad" -o run --output-format csv -- python3 tools/bench_grad.py --reps 3 --only gram,kuf,kuf_incr,pde,pde_gram,sig,svgp46,svgp126,vosf_kdiag > "$OUT/grad_prof.log" 2>&1 || exit 4
timeout -k 10 900 python3 tools/bench_grad.py --reps 5 --only gram,kuf,kuf_incr,pde,pde_gram,sig,svgp46,svgp126,vosf_kdiag > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 5
