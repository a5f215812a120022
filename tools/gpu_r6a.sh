#!/bin/bash
# Round 6 (a): the TF-bridge host bodies and the reworked gradient assertions on the GPU; C4 / C4i counters
# (one rocprofv3 --pmc pass per counter group) for C4's physical roofline.
set -o pipefail
OUT=gpurun_out/r6a
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tf_bridge_gpu.py \
  "tests/test_grad_gpu.py::test_gram_vjp_shapes" "tests/test_ho_grad_gpu.py::test_higher_order_signature_kernel_gradient" \
  > "$OUT/tests.log" 2>&1 || exit 1
F32="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
WAIT="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
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
