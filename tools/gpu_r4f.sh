#!/bin/bash
# Matrix-core wide Gram with column blocks: parity, and timings against the runtime channel loop.
OUT=${1:-gpurun_out/r4f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_grad_gpu.py tests/test_long_gpu.py tests/test_long_grad_gpu.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
r=$?; tail -3 "$OUT/pytest.log"; [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
timeout -k 10 300 python -u tools/bench_wide.py --l 500 --n 256 --d 46 126 > "$OUT/mf_l500.jsonl" 2>&1 || exit $?
GPSIG_WIDE_MF=0 timeout -k 10 300 python -u tools/bench_wide.py --l 500 --n 256 --d 46 126 > "$OUT/loop_l500.jsonl" 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_wide.py --l 136 --d 46 126 > "$OUT/mf_l136.jsonl" 2>&1 || exit $?
grep -h '"n"' "$OUT"/*.jsonl
timeout -k 10 300 python -u -m pytest tests/test_wide_gpu.py -m gpu -v -k "higher_order or mf_column" --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_ho.log" 2>&1
tail -3 "$OUT/pytest_ho.log"
