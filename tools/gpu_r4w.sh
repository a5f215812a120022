#!/bin/bash
# Round-4 close after the GEMM rework: the full GPU suite + smoke + bench, then the SVGP step's kernel
# trace (rocprofv3 --kernel-trace --stats) at D = 126.
bash tools/gpu_suite.sh gpurun_out/r4suite3 || exit $?
OUT=gpurun_out/r4w
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_svgp126" -o run --output-format csv -- python3 tools/bench_grad.py --only svgp126 --reps 3 > "$OUT/prof_svgp126.log" 2>&1 || exit $?
grep -h "^{" "$OUT/prof_svgp126.log"
