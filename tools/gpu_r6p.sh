#!/bin/bash
# Round 6 (p): split-f16 generic GEMM: the GPU suite, the SVGP step and the P128 row with traces, and the
# same with GPSIG_GEMM_F16=0 (f32 kernel) for A/B.
set -o pipefail
OUT=gpurun_out/r6p
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/svgp" -o run --output-format csv -- \
  python3 tools/bench_grad.py --only svgp46,svgp126 > "$OUT/svgp.jsonl" 2> "$OUT/svgp.err" || exit 2
GPSIG_GEMM_F16=0 timeout -k 10 300 python3 tools/bench_grad.py --only svgp46,svgp126 > "$OUT/svgp_f32.jsonl" 2> "$OUT/svgp_f32.err" || exit 3
timeout -k 10 300 python3 tools/bench_rows.py --rows P128 --reps 5 --cpu-seconds 0.2 > "$OUT/p128.jsonl" 2> "$OUT/p128.err" || exit 4
GPSIG_GEMM_F16=0 timeout -k 10 300 python3 tools/bench_rows.py --rows P128 --reps 5 --cpu-seconds 0.2 > "$OUT/p128_f32.jsonl" 2> "$OUT/p128_f32.err" || exit 5
exit 0
