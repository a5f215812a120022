#!/bin/bash
# A/B of the RBF seed engine of the headline Gram kernel (packed VALU dots vs v_mfma_f32_4x4x1f32),
# at H (N=4096, L=128, D=5, M=5) and C5 on one GPU (N=8192, L=128, D=8, M=6), plus one SQ counter pass of
# each arm at H.  Run on the GPU box from the repo root:  tools/ab_seed.sh gpurun_out/ab
OUT=${1:-gpurun_out/ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in H C5; do
  for eng in valu mfma; do
    steps=5; [ $wl = C5 ] && steps=2
    timeout -k 10 240 python3 -u bench.py --workload $wl --seed-engine $eng --steps $steps --warmup 1 --no-cpu --no-probe \
      > "$OUT/bench_${wl}_${eng}.json" 2> "$OUT/bench_${wl}_${eng}.err" || exit 1
    cat "$OUT/bench_${wl}_${eng}.json"
  done
done
for eng in valu mfma; do
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE \
    -d "$OUT/sq_$eng" -o run --output-format csv -- python3 bench.py --seed-engine $eng --steps 2 --warmup 1 --no-cpu --no-check --no-probe \
    > "$OUT/sq_$eng.log" 2>&1 || exit 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr_$eng" -o run --output-format csv -- python3 bench.py --seed-engine $eng --steps 2 --warmup 1 --no-cpu --no-check --no-probe \
    > "$OUT/tr_$eng.log" 2>&1 || exit 3
done
exit 0
