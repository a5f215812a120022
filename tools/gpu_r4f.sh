#!/bin/bash
# Matrix-core wide Gram with column blocks: parity, and timings against the runtime channel loop.
OUT=${1:-gpurun_out/r4f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ho_grad_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_hograd.log" 2>&1
r=$?; tail -3 "$OUT/pytest_hograd.log"; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_long_gpu.py tests/test_long_grad_gpu.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
r=$?; tail -3 "$OUT/pytest.log"; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 300 python -u tools/bench_wide.py --l 500 --n 256 --d 46 126 > "$OUT/mf_l500.jsonl" 2>&1 || exit $?
GPSIG_WIDE_MF=0 timeout -k 10 300 python -u tools/bench_wide.py --l 500 --n 256 --d 46 126 > "$OUT/loop_l500.jsonl" 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_wide.py --l 136 --d 46 126 > "$OUT/mf_l136.jsonl" 2>&1 || exit $?
grep -h '"n"' "$OUT"/*.jsonl
timeout -k 10 300 python -u -m pytest tests/test_wide_gpu.py -m gpu -v -k "higher_order or mf_column" --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_ho.log" 2>&1
tail -3 "$OUT/pytest_ho.log"
for D in 46 126; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_svgp$D" -o run --output-format csv -- python3 tools/bench_grad.py --only svgp$D --reps 2 > "$OUT/prof_svgp$D.log" 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob
for D in (46, 126):
    f = glob.glob(f"gpurun_out/r4f/prof_svgp{D}/**/run_kernel_stats.csv", recursive=True)
    if not f: print("no stats", D); continue
    rows = list(csv.DictReader(open(f[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("svgp", D, "total ms", tot / 1e6)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
        print("  %-90s calls %5s total %8.2f ms  %4.1f%%" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e6, 100 * float(r["TotalDurationNs"]) / tot))
PY
