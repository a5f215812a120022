#!/bin/bash
# Round 5 headline evidence: the default bench line, its rocprofv3 kernel trace, and the PMC passes
# (profiles/run_profile.sh), plus the rows' traces.
set -o pipefail
OUT=gpurun_out/r5l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 900 bash profiles/run_profile.sh $OUT/prof || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/rows" -o run --output-format csv -- python3 tools/bench_rows.py --rows C2,C3,C4,C4i,C5,W46,W126 --reps 3 --cpu-seconds 1 --out "$OUT/rows_prof.json" > "$OUT/rows_prof.log" 2>&1 || exit 3
timeout -k 10 600 python3 tools/bench_rows.py --rows C2,C3,C4,C4i,C5,W46,W126 --reps 5 --cpu-seconds 2 --out "$OUT/rows.json" > "$OUT/rows.log" 2>&1 || exit 4
