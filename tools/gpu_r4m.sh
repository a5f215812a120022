#!/bin/bash
# Wide diagonal forward on seed tiles + tensor-Gram forward on pair tiles: parity, SVGP / VOSF-Kdiag timing.
OUT=${1:-gpurun_out/r4m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_tensors_gpu.py tests/test_training_gpu.py tests/test_ho_grad_gpu.py tests/test_full_size_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
r=$?; tail -3 "$OUT/pytest.log"; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
for D in 46 126; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_svgp$D" -o run --output-format csv -- python3 tools/bench_grad.py --only svgp$D --reps 3 > "$OUT/prof_svgp$D.log" 2>&1 || exit $?
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_vosf" -o run --output-format csv -- python3 tools/bench_grad.py --only vosf_kdiag --reps 3 > "$OUT/vosf.jsonl" 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.5 --out "$OUT/rows.json" > "$OUT/rows.log" 2>&1 || exit $?
cat "$OUT"/svgp*.jsonl; grep "^{" "$OUT/vosf.jsonl"
python3 - <<'PY'
import csv, glob, json
for tag in ("svgp46", "svgp126", "vosf"):
    f = glob.glob(f"gpurun_out/r4m/prof_{tag}/**/run_kernel_stats.csv", recursive=True)
    if not f: print("no stats", tag); continue
    rows = list(csv.DictReader(open(f[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(tag, "total ms", tot / 1e6)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
        print("  %-90s calls %5s total %8.2f ms  %4.1f%%" % (r["Name"][:90], r["Calls"], float(r["TotalDurationNs"]) / 1e6, 100 * float(r["TotalDurationNs"]) / tot))
for r in json.load(open("gpurun_out/r4m/rows.json")):
    print(r["config"], r["ms_per_call"], r["gram_kernel_ms"], r["max_abs_err"])
PY
