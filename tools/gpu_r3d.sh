# Round-3 evidence: the MFMA seed A/B on the kept kernel (tools/ab_seed.sh), kernel traces and SQ busy
# counters of the SURVEY 8 rows C2 / C3 / W126, and of the Gram VJP (register form; tile form with GEMMs).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
PMC="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
bash tools/ab_seed.sh $O/ab || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rows_trace -o run --output-format csv -- python3 tools/bench_rows.py --rows C2,C3,W126 --reps 3 --cpu-seconds 0.5 > $O/rows_trace.log 2>&1 || exit 2
for r in C2 C3 W126; do
  timeout -s KILL 180 rocprofv3 --pmc $PMC -d $O/pmc_$r -o run --output-format csv -- python3 tools/bench_rows.py --rows $r --reps 1 --cpu-seconds 0.5 > $O/pmc_$r.log 2>&1 || exit 3
done
timeout -s KILL 180 rocprofv3 --pmc $PMC -d $O/pmc_vjp -o run --output-format csv -- python3 tools/bench_grad.py --only gram --reps 2 > $O/pmc_vjp.log 2>&1 || exit 4
GPSIG_VJP_FIXED_MAX=0 timeout -s KILL 180 rocprofv3 --pmc $PMC -d $O/pmc_vjp_tile -o run --output-format csv -- python3 tools/bench_grad.py --only gram --reps 2 > $O/pmc_vjp_tile.log 2>&1 || exit 5
exit 0
