#!/bin/bash
# DIAG seed tiles of the wide VJP (Kff diagonal): parity, observed gradient errors, SVGP profile; then the
# matrix-core Gram at the fixed channel counts (A/B, tools/gpu_r4k.sh).
OUT=${1:-gpurun_out/r4l}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_training_gpu.py tests/test_ho_grad_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
r=$?; tail -3 "$OUT/pytest.log"; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 300 python3 tools/grad_err_scan.py > "$OUT/grad_err.log" 2>&1; tail -40 "$OUT/grad_err.log" | grep max_norm
for D in 46 126; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_svgp$D" -o run --output-format csv -- python3 tools/bench_grad.py --only svgp$D --reps 3 > "$OUT/prof_svgp$D.log" 2>&1 || exit $?
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
cat "$OUT"/svgp*.jsonl
python3 - <<'PY'
import csv, glob
for D in (46, 126):
    f = glob.glob(f"gpurun_out/r4l/prof_svgp{D}/**/run_kernel_stats.csv", recursive=True)
    if not f: print("no stats", D); continue
    rows = list(csv.DictReader(open(f[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("svgp", D, "total ms", tot / 1e6)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
        print("  %-90s calls %5s total %8.2f ms  %4.1f%%" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e6, 100 * float(r["TotalDurationNs"]) / tot))
PY
bash tools/gpu_r4k.sh gpurun_out/r4k
