#!/bin/bash
# Build the Gram-VJP A/B variants (tools/kbench_vjp.hip) into tools/bin/.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -mllvm -amdgpu-atomic-optimizer-strategy=None"
b() { name=$1; shift; hipcc $F -DVARIANT=\"$name\" "$@" tools/kbench_vjp.hip -o tools/bin/$name & }
b v_base
b v_noemit -DGPSIG_BWD_ABL=1
b v_noinv -DGPSIG_BWD_ABL=2
b v_noadj -DGPSIG_BWD_ABL=4
b v_none -DGPSIG_BWD_ABL=7
wait
ls tools/bin
