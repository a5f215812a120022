#!/bin/bash
# A/B of the MF kernel's K padding (KQ = 2 mod 4 vs the smallest even KQ) on the wide rows + parity.
OUT=${1:-gpurun_out/r4p}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.2 --out "$OUT/kq1.json" > "$OUT/kq1.log" 2>&1 || exit $?
GPSIG_MF_KQ=0 timeout -k 10 300 python3 tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 0.2 --out "$OUT/kq0.json" > "$OUT/kq0.log" 2>&1 || exit $?
GPSIG_MF_KQ=0 timeout -k 10 300 python -u -m pytest tests/test_wide_gpu.py -m gpu -q -k "wide_rbf_gram or mf_column or normalised" --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_kq0.log" 2>&1
tail -2 "$OUT/pytest_kq0.log"
python3 - <<'PY'
import json
for f in ("kq1", "kq0"):
    for r in json.load(open(f"gpurun_out/r4p/{f}.json")):
        print(f, r["config"], round(r["gram_kernel_ms"], 2), r["max_abs_err"])
PY
