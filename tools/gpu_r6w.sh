#!/bin/bash
# Round 6 (w): signature VJP with its global loads one step ahead (measured no faster, reverted): bench row and trace.
set -o pipefail
OUT=gpurun_out/r6w
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 python3 tools/bench_grad.py --only sig >> "$OUT/sig.txt" 2>&1 || exit 2
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 tools/bench_grad.py --only sig > "$OUT/trace.log" 2>&1 || exit 3
exit 0
