# Round-3 (session 2): parity of the 10-lane forward / 20-lane VJP geometries, then the C2 row and the
# gradient table.  Each GPU step has its own limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gram_gpu.py tests/test_grad_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u tools/bench_rows.py --rows C2 --reps 5 --cpu-seconds 1 --out $O/rows_c2.json > $O/rows.log 2>&1 || { tail -20 $O/rows.log; exit 2; }
timeout -k 10 300 python -u tools/bench_grad.py --only gram --reps 5 > $O/grad.jsonl 2> $O/grad.err || { tail -20 $O/grad.err; exit 3; }
cat $O/grad.jsonl
exit 0
