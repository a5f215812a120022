#!/bin/bash
# Round 6 (z): headline profile passes and bench line on the final tree (anchor period 128).
set -o pipefail
OUT=gpurun_out/r6z
mkdir -p "$OUT"
export TMPDIR=/tmp
bash profiles/run_profile.sh "$OUT/prof" || exit 1
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 2
exit 0
