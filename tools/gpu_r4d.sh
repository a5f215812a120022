#!/bin/bash
OUT=${1:-gpurun_out/r4d}
mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in "--l 161 --m 2" "--l 300 --m 4 --base linear" "--l 300 --m 4" "--l 500 --l2 493 --m 4"; do
  tag=$(echo $cfg | tr -d ' -')
  GPSIG_WIDE_MF_BLK=1 timeout -k 10 120 python -u tools/diag_mf.py "$OUT/mf_$tag.npz" $cfg || exit $?
  GPSIG_WIDE_MF=0 timeout -k 10 120 python -u tools/diag_mf.py "$OUT/loop_$tag.npz" $cfg || exit $?
done
python - <<'PY'
import glob, numpy as np
for f in sorted(glob.glob("gpurun_out/r4d/mf_*.npz")):
    a, b = np.load(f), np.load(f.replace("/mf_", "/loop_"))
    for k in ("rect", "sym"):
        x, y = a[k], b[k]
        print(f, k, [float(np.abs(x[m] - y[m]).max() / max(np.abs(y[m]).max(), 1e-30)) for m in range(x.shape[0])])

PY
