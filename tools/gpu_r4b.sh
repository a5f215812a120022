#!/bin/bash
# Round 4: matrix-core wide-channel Gram -- parity (wide tests) and the A/B against the runtime channel loop;
# the slot-invariant segmented scan (C2 bitwise subset test + C2 timing); the SVGP step rows.
OUT=${1:-gpurun_out/r4b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_full_size_gpu.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
r=$?; tail -5 "$OUT/pytest.log"; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 300 python -u tools/bench_wide.py --l 128 --d 16 32 46 126 > "$OUT/mf_l128.jsonl" 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_wide.py --l 136 --d 46 > "$OUT/mf_l136.jsonl" 2>&1 || exit $?
GPSIG_WIDE_MF=0 timeout -k 10 300 python -u tools/bench_wide.py --l 128 --d 16 46 126 > "$OUT/loop_l128.jsonl" 2>&1 || exit $?
cat "$OUT"/*.jsonl
timeout -k 10 300 python -u tools/bench_rows.py --rows C2 --cpu-seconds 1 > "$OUT/c2.json" 2>&1 || exit $?
tail -2 "$OUT/c2.json"
timeout -k 10 300 python -u tools/bench_grad.py --only gram,svgp46,svgp126 --reps 3 > "$OUT/grad.jsonl" 2>&1 || exit $?
cat "$OUT/grad.jsonl"
