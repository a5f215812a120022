#!/bin/bash
# Round-4 closing run: the full GPU suite + smoke + bench (tools/gpu_suite.sh), the SVGP timing with the
# Kuf seed prefetch, then the MF K-padding A/B (tools/gpu_r4p.sh).
bash tools/gpu_suite.sh gpurun_out/r4suite2 || exit $?
OUT=gpurun_out/r4r
mkdir -p "$OUT"
export TMPDIR=/tmp
for D in 46 126; do
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
cat "$OUT"/svgp*.jsonl | grep "^{"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_svgp126" -o run --output-format csv -- python3 tools/bench_grad.py --only svgp126 --reps 3 > "$OUT/prof_svgp126.log" 2>&1 || exit $?
bash tools/gpu_r4p.sh gpurun_out/r4p
