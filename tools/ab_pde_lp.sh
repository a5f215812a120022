# PDE lane-group A/B at C3 (N = 1024, L = 200, dyadic 1): the cost model's pick vs LP pinned to 32 / 16.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_pde_lp
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pde_gpu.py tests/test_pde_grad.py tests/test_long_gpu.py -q -k pde --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 200 python3 -u tools/bench_rows.py --rows C3 --cpu-seconds 0.5 > $O/c3_auto.log 2>&1 || exit 2
GPSIG_PDE_LP=32 timeout -k 10 200 python3 -u tools/bench_rows.py --rows C3 --cpu-seconds 0.5 > $O/c3_lp32.log 2>&1 || exit 3
GPSIG_PDE_LP=16 timeout -k 10 200 python3 -u tools/bench_rows.py --rows C3 --cpu-seconds 0.5 > $O/c3_lp16.log 2>&1 || exit 4
grep -h '^{' $O/c3_*.log
