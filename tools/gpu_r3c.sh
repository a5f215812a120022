# Full GPU suite after the forward crossover change, then the wide-channel rows and the gradient A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
r=$?; tail -15 $O/pytest.log; [ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 300 python3 -u tools/bench_wide.py --d 5 8 12 16 26 32 46 126 > $O/wide.jsonl 2>&1 || exit 2
cat $O/wide.jsonl
timeout -k 10 300 python3 -u tools/bench_rows.py --rows W46,W126 --out $O/rows_wide.json > $O/rows_wide.log 2>&1 || exit 3
cat $O/rows_wide.log
exit 0
