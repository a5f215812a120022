set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 1000 python -u -m pytest tests/test_wide_gpu.py tests/test_gemm_gpu.py tests/test_pde_wide_gpu.py tests/test_long_gpu.py tests/test_pde_gpu.py tests/test_pde_grad.py tests/test_gram_gpu.py tests/test_grad_gpu.py tests/test_ho_grad_gpu.py tests/test_distributed.py --maxfail=40 -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a/pytest.log 2>&1
r=$?; tail -45 gpurun_out/r3a/pytest.log; [ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 300 python -u tools/bench_wide.py --d 8 16 32 46 126 > gpurun_out/r3a/wide.jsonl 2>&1 || exit $?
GPSIG_FO_FIXED_MAX=0 timeout -k 10 300 python -u tools/bench_wide.py --d 5 8 16 32 > gpurun_out/r3a/wide_forced.jsonl 2>&1 || exit $?
cat gpurun_out/r3a/wide.jsonl gpurun_out/r3a/wide_forced.jsonl
timeout -k 10 300 python -u tools/bench_grad.py --only gram > gpurun_out/r3a/grad_fixed.jsonl 2>&1 || exit $?
GPSIG_VJP_FIXED_MAX=0 timeout -k 10 300 python -u tools/bench_grad.py --only gram > gpurun_out/r3a/grad_wide.jsonl 2>&1 || exit $?
cat gpurun_out/r3a/grad_fixed.jsonl gpurun_out/r3a/grad_wide.jsonl
