# Round-3 measurements on one MI355X: the PDE parity tests (lane-group geometry change), the headline
# bench + its kernel trace, the SURVEY 8 rows (with the wide-channel rows), the gradient paths, and one
# SQ counter pass of the wide-channel Gram row.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_pde_gpu.py tests/test_pde_grad.py tests/test_pde_wide_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pde_tests.log 2>&1
r=$?; tail -3 $O/pde_tests.log; [ $r -ne 0 ] && [ $r -ne 1 ] && exit $r
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-check --no-probe > $O/trace.log 2>&1 || exit 2
timeout -k 10 600 python3 -u tools/bench_rows.py --rows C2,C3,C4,C4i,C5,W46,W126,P128 --out $O/rows.json > $O/rows.log 2>&1 || exit 3
cat $O/rows.log
timeout -k 10 400 python3 -u tools/bench_grad.py > $O/grad.jsonl 2>&1 || exit 4
cat $O/grad.jsonl
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_w126 -o run --output-format csv -- python3 tools/bench_rows.py --rows W126 --reps 1 --cpu-seconds 0.5 > $O/pmc_w126.log 2>&1 || exit 5
exit 0
