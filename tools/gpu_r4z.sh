#!/bin/bash
# Round-4: Kuf forward timing in the small-increment and corner regimes, previous kernel
# (gpsig_amd/_ab/libgpsig_old.so) vs the corner differences off the exact pass and the seeds.
OUT=${1:-gpurun_out/r4z}
mkdir -p "$OUT"
export TMPDIR=/tmp
GPSIG_AMD_LIB=gpsig_amd/_ab/libgpsig_old.so timeout -k 10 300 python3 tools/bench_kuf_corner.py > "$OUT/kuf_old.jsonl" 2>&1 || exit $?
timeout -k 10 300 python3 tools/bench_kuf_corner.py > "$OUT/kuf_new.jsonl" 2>&1 || exit $?
grep -h "^{" "$OUT"/kuf_old.jsonl "$OUT"/kuf_new.jsonl
