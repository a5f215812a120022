set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 900 python -u -m pytest tests/test_wide_gpu.py tests/test_gemm_gpu.py tests/test_pde_wide_gpu.py tests/test_pde_gpu.py tests/test_pde_grad.py tests/test_gram_gpu.py tests/test_grad_gpu.py --maxfail=40 -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a/pytest.log 2>&1
r=$?; tail -45 gpurun_out/r3a/pytest.log; [ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 300 python -u tools/bench_wide.py --d 8 16 32 46 126 > gpurun_out/r3a/wide.jsonl 2>&1 || exit $?
GPSIG_FO_FIXED_MAX=0 timeout -k 10 300 python -u tools/bench_wide.py --d 5 8 16 32 > gpurun_out/r3a/wide_forced.jsonl 2>&1 || exit $?
cat gpurun_out/r3a/wide.jsonl gpurun_out/r3a/wide_forced.jsonl
