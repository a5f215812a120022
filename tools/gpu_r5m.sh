#!/bin/bash
# Round 5 counters of the rows (one --pmc pass each) and the gradient benchmark with its trace
OUT=gpurun_out/r5m
mkdir -p "$OUT"
export TMPDIR=/tmp
F32="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
pmc() {  # name rows counters...
  local name=$1 rows=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/pmc_$name" -o run --output-format csv -- python3 tools/bench_rows.py --rows $rows --reps 1 --cpu-seconds 0.2 > "$OUT/pmc_$name.log" 2>&1 || return 1
  python3 tools/sq_busy.py "$OUT/pmc_$name" > "$OUT/pmc_$name.json" || return 2
}
pmc c2_f32 C2 $F32 || exit 11
pmc c5_f32 C5 $F32 || exit 12
pmc w46_mf W46 $MF || exit 13
pmc w126_mf W126 $MF || exit 14
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/grad" -o run --output-format csv -- python3 tools/bench_grad.py --reps 3 --only gram,pde_gram,vosf_kdiag > "$OUT/grad_prof.log" 2>&1 || exit 15
timeout -k 10 900 python3 tools/bench_grad.py --reps 5 --only gram,kuf,kuf_incr,pde,pde_gram,sig,svgp46,svgp126,vosf_kdiag > "$OUT/grad.jsonl" 2> "$OUT/grad.err" || exit 16
