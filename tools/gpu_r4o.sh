#!/bin/bash
# Backward-path timings of round 4 (tools/bench_grad.py default set + the SVGP / VOSF rows) and the kernel
# trace of the Gram and PDE-Gram rows.
OUT=${1:-gpurun_out/r4o}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/bench_grad.py --reps 5 --only gram,kuf,kuf_incr,pde,pde_gram,sig,svgp46,svgp126,vosf_kdiag > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit $?
cat "$OUT/grad.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_gram" -o run --output-format csv -- python3 tools/bench_grad.py --only gram,pde_gram --reps 3 > "$OUT/prof_gram.log" 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r4o/prof_gram/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("  %-100s calls %5s avg %8.3f ms" % (r["Name"][:100], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
