#!/bin/bash
# Round-4 A/B of the LDS-state higher-order VJP: slab loads behind a per-load memory clobber (in-tree lib)
# vs. a laundered slab pointer per load (gpsig_amd/_ab/libgpsig_launder.so, -DHO_LAUNDER): parity of both on
# tests/test_ho_grad_gpu.py, then the VOSF order-5 Kdiag timing; finally the wide/MF tests that cover the
# reverted Kuf prefetch and the removed MF K-padding switch.
OUT=${1:-gpurun_out/r4s}
mkdir -p "$OUT"
export TMPDIR=/tmp
T="python3 -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_ho_grad_gpu.py > "$OUT/ho_default.log" 2>&1 || exit $?
tail -1 "$OUT/ho_default.log"
GPSIG_AMD_LIB=gpsig_amd/_ab/libgpsig_launder.so timeout -k 10 600 $T tests/test_ho_grad_gpu.py > "$OUT/ho_launder.log" 2>&1 || exit $?
tail -1 "$OUT/ho_launder.log"
timeout -k 10 300 python3 tools/bench_grad.py --only vosf_kdiag --reps 10 > "$OUT/vosf_default.jsonl" 2>&1 || exit $?
GPSIG_AMD_LIB=gpsig_amd/_ab/libgpsig_launder.so timeout -k 10 300 python3 tools/bench_grad.py --only vosf_kdiag --reps 10 > "$OUT/vosf_launder.jsonl" 2>&1 || exit $?
grep -h "^{" "$OUT"/vosf_*.jsonl
timeout -k 10 600 $T tests/test_wide_gpu.py > "$OUT/wide.log" 2>&1 || exit $?
tail -1 "$OUT/wide.log"
for D in 46 126; do
  timeout -k 10 300 python3 tools/bench_grad.py --only svgp$D --reps 5 > "$OUT/svgp$D.jsonl" 2>&1 || exit $?
done
grep -h "^{" "$OUT"/svgp*.jsonl
