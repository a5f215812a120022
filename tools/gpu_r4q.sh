#!/bin/bash
# Kuf seed prefetch (forward two steps ahead, VJP one): parity and SVGP timing.
OUT=${1:-gpurun_out/r4q}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_tensors_gpu.py tests/test_training_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
r=$?; tail -3 "$OUT/pytest.log"; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
for D in 46 126; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_svgp$D" -o run --output-format csv -- python3 tools/bench_grad.py --only svgp$D --reps 3 > "$OUT/prof_svgp$D.log" 2>&1 || exit $?
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
cat "$OUT"/svgp*.jsonl | grep "^{"
python3 - <<'PY'
import csv, glob
for D in (46, 126):
    f = glob.glob(f"gpurun_out/r4q/prof_svgp{D}/**/run_kernel_stats.csv", recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:6]:
        print(D, "  %-80s calls %5s avg %8.3f ms" % (r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
