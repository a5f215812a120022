#!/bin/bash
# Round-4 closing run on the final tree: the full GPU suite + smoke + bench, the SVGP step timing, and the
# VOSF / Kuf corner rows.
bash tools/gpu_suite.sh gpurun_out/r4suite4 || exit $?
OUT=gpurun_out/r4zb
mkdir -p "$OUT"
export TMPDIR=/tmp
for D in 46 126; do
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
grep -h "^{" "$OUT"/svgp*.jsonl
