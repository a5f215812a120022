#!/bin/bash
# Round 6 (b): the packed column-pair Gram VJP (sig_bwd_pk.h) -- gradient suites, then fwd+bwd A/B against
# the round-5 kernel (GPSIG_BWD_PK=0) at C2's shape, then the C4 / C4i counters left from r6a.
set -o pipefail
OUT=gpurun_out/r6b
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ho_grad_gpu.py \
  > "$OUT/grad_tests.log" 2>&1 || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_long_grad_gpu.py \
  tests/test_training_gpu.py tests/test_tf_bridge_gpu.py > "$OUT/more_tests.log" 2>&1 || exit 2
GPSIG_BWD_PK=0 timeout -k 10 300 python3 tools/bench_grad.py --reps 5 --only gram > "$OUT/gram_r5kernel.jsonl" 2> "$OUT/gram_r5kernel.err" || exit 3
timeout -k 10 300 python3 tools/bench_grad.py --reps 5 --only gram > "$OUT/gram_pk.jsonl" 2> "$OUT/gram_pk.err" || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/gramtrace" -o run --output-format csv -- python3 tools/bench_grad.py --reps 3 --only gram > "$OUT/gramtrace.log" 2>&1 || exit 5
F32="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
WAIT="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $F32 -d "$OUT/pmc_gram_f32" -o run --output-format csv -- python3 tools/bench_grad.py --reps 1 --only gram > "$OUT/pmc_gram_f32.log" 2>&1 || exit 6
python3 tools/sq_busy.py "$OUT/pmc_gram_f32" sig_bwd > "$OUT/pmc_gram_f32.json" || exit 7
pmc() {  # name rows counters...
  local name=$1 rows=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/pmc_$name" -o run --output-format csv -- python3 tools/bench_rows.py --rows $rows --reps 1 --cpu-seconds 0.2 > "$OUT/pmc_$name.log" 2>&1 || return 1
  python3 tools/sq_busy.py "$OUT/pmc_$name" > "$OUT/pmc_$name.json" || return 2
}
for row in C4 C4i; do
  pmc ${row}_f32 $row $F32 || exit 11
  pmc ${row}_wait $row $WAIT || exit 12
  pmc ${row}_fetch $row FETCH_SIZE GRBM_GUI_ACTIVE || exit 13
  pmc ${row}_write $row WRITE_SIZE GRBM_GUI_ACTIVE || exit 14
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/c4trace" -o run --output-format csv -- python3 tools/bench_rows.py --rows C4,C4i --reps 3 --cpu-seconds 0.2 > "$OUT/c4trace.log" 2>&1 || exit 15
