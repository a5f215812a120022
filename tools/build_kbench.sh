#!/bin/bash
# Build the kbench A/B variants (tools/kbench.hip) into tools/bin/.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize"
b() { name=$1; shift; hipcc $F -DVARIANT=\"$name\" "$@" tools/kbench.hip -o tools/bin/$name & }
b g_w4 -DKW=4 -DKLP=32
b g_w8 -DKW=8 -DKLP=16
b g_w8_nn -DKW=8 -DKLP=16 -DGPSIG_NAIVE=0
wait
ls tools/bin
