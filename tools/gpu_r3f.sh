# Round-3 (session 2) evidence after the segmented lane groups: the whole GPU suite, smoke, the headline
# bench, rocprofv3 kernel traces of the bench / C2 row / Gram training step, and SQ busy counters of C2's
# Gram launch and the Gram VJP.  Each GPU step has its own limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
PMC="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
bash tools/gpu_suite.sh $O/suite || exit 1
bash profiles/run_profile.sh $O/prof || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rows_trace -o run --output-format csv -- python3 tools/bench_rows.py --rows C2 --reps 3 --cpu-seconds 0.5 > $O/rows_trace.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/grad_trace -o run --output-format csv -- python3 tools/bench_grad.py --only gram --reps 3 > $O/grad_trace.log 2>&1 || exit 4
timeout -s KILL 180 rocprofv3 --pmc $PMC -d $O/pmc_c2 -o run --output-format csv -- python3 tools/bench_rows.py --rows C2 --reps 1 --cpu-seconds 0.5 > $O/pmc_c2.log 2>&1 || exit 5
timeout -s KILL 180 rocprofv3 --pmc $PMC -d $O/pmc_vjp -o run --output-format csv -- python3 tools/bench_grad.py --only gram --reps 2 > $O/pmc_vjp.log 2>&1 || exit 6
timeout -k 10 300 python -u tools/bench_rows.py --rows C2 --reps 5 --cpu-seconds 5 --out $O/rows_c2.json > $O/rows.log 2>&1 || exit 7
timeout -k 10 300 python -u tools/bench_grad.py --reps 5 > $O/grad.jsonl 2> $O/grad.err || exit 8
cat $O/grad.jsonl
exit 0
