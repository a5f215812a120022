#!/bin/bash
# MF column-block diagnostic (A/B vs the runtime channel loop) and the seg-scan retest.
OUT=${1:-gpurun_out/r4c}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "--l 161 --m 2" "--l 300 --m 2" "--l 300 --m 4" "--l 300 --m 4 --base linear" "--l 161 --l2 140 --m 3"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 120 python -u tools/diag_mf.py "$OUT/mf_$tag.npz" $cfg || exit $?
  GPSIG_WIDE_MF=0 timeout -k 10 120 python -u tools/diag_mf.py "$OUT/loop_$tag.npz" $cfg || exit $?
done
python - <<'PY'
import glob, numpy as np
for f in sorted(glob.glob("gpurun_out/r4c/mf_*.npz")):
    a, b = np.load(f), np.load(f.replace("/mf_", "/loop_"))
    for k in ("rect", "sym"):
        x, y = a[k], b[k]
        print(f, k, [float(np.abs(x[m] - y[m]).max() / max(np.abs(y[m]).max(), 1e-30)) for m in range(x.shape[0])])
PY
timeout -k 10 600 python -u -m pytest tests/test_grad_gpu.py tests/test_full_size_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "twenty or full_size" > "$OUT/pytest.log" 2>&1
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u tools/bench_rows.py --rows C2 --cpu-seconds 1 > "$OUT/c2.json" 2>&1 || exit $?
tail -1 "$OUT/c2.json"
