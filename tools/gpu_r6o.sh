#!/bin/bash
# Round 6 (o): the SVGP training step at D = 46 / 126 with a kernel trace (where the time goes).
set -o pipefail
OUT=gpurun_out/r6o
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/svgp" -o run --output-format csv -- \
  python3 tools/bench_grad.py --only svgp46,svgp126 > "$OUT/svgp.jsonl" 2> "$OUT/svgp.err" || exit 1
