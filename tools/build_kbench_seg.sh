#!/bin/bash
# Segmented-scan radix A/B (common.h seg_incl_scan_n, GPSIG_SEG_RADIX 2 vs 4) on the kernels that use it at C2's
# shape: the 10-lane Gram forward (tools/kbench.hip) and the 20-lane round-5 VJP (tools/kbench_vjp.hip).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize"
b() { src=$1; name=$2; shift 2; /opt/rocm/bin/hipcc $F -DVARIANT=\"$name\" "$@" tools/$src.hip -o tools/bin/$name & }
b kbench c2f_r2 -DKL=100 -DKW=10 -DKLP=10 -DGPSIG_SEG_RADIX=2
b kbench c2f_r4 -DKL=100 -DKW=10 -DKLP=10 -DGPSIG_SEG_RADIX=4
b kbench_vjp c2b_r2 -DKW=5 -DKLP=20 -DKSTATE=1 -DGPSIG_SEG_RADIX=2 -mllvm -amdgpu-atomic-optimizer-strategy=None
b kbench_vjp c2b_r4 -DKW=5 -DKLP=20 -DKSTATE=1 -DGPSIG_SEG_RADIX=4 -mllvm -amdgpu-atomic-optimizer-strategy=None
wait
