#!/bin/bash
# A/B: the matrix-core Gram kernel (sig_fo_mf.h) at the fixed channel counts (GPSIG_FO_FIXED_MAX below d
# routes d to the wide path) against the fixed-channel VALU kernels: C2 (D=5, L=100), C5 (D=8, L=128), H.
OUT=${1:-gpurun_out/r4k}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_rows.py --rows C2,C5 --reps 3 --cpu-seconds 0.2 --out "$OUT/valu.json" > "$OUT/valu.log" 2>&1 || exit $?
GPSIG_FO_FIXED_MAX=4 timeout -k 10 300 python3 tools/bench_rows.py --rows C2,C5 --reps 3 --cpu-seconds 0.2 --out "$OUT/mf.json" > "$OUT/mf.log" 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > "$OUT/h_valu.json" 2> "$OUT/h_valu.err" || exit $?
GPSIG_FO_FIXED_MAX=4 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 > "$OUT/h_mf.json" 2> "$OUT/h_mf.err" || exit $?
python3 - <<'PY'
import json
for f in ("valu", "mf"):
    for r in json.load(open(f"gpurun_out/r4k/{f}.json")):
        print(f, r["config"], round(r["gram_kernel_ms"], 2), round(r["roofline"]["frac"], 3), r["max_abs_err"])
for f in ("h_valu", "h_mf"):
    l = [x for x in open(f"gpurun_out/r4k/{f}.json") if x.startswith("{")][-1]
    r = json.loads(l)
    print(f, r["value"], r["ms_per_step"], r["roofline"]["frac"], r.get("max_abs_err"))
PY
