# Wide-channel forward with the LDS-DMA staged channel loop: parity (wide, long, Gram, grad, distributed
# suites that reach the wide kernels), then the wide rows.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_long_gpu.py tests/test_gram_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u tools/bench_wide.py --d 16 32 46 126 > $O/wide.jsonl 2> $O/wide.err || { tail -20 $O/wide.err; exit 2; }
cat $O/wide.jsonl
timeout -k 10 300 python -u tools/bench_rows.py --rows W46,W126 --reps 5 --cpu-seconds 1 --out $O/rows_w.json > $O/rows.log 2>&1 || { tail -20 $O/rows.log; exit 3; }
exit 0
