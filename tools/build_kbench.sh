#!/bin/bash
# Build the kbench A/B variants (tools/kbench.hip) into tools/bin/.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize"
b() { name=$1; shift; hipcc $F -DVARIANT=\"$name\" "$@" tools/kbench.hip -o tools/bin/$name & }
b g_w4 -DKW=4 -DKLP=32
b g_w8 -DKW=8 -DKLP=16
# MFMA seed (RbfSeedPk::mfma_pc) A/B
b g_w4_mf -DKW=4 -DKLP=32 -DKMF=1
b g_w4_mf_lb3 -DKW=4 -DKLP=32 -DKMF=1 -DGPSIG_FO_LB=3
b g_w8_mf -DKW=8 -DKLP=16 -DKMF=1
b g_w8_mf_lb2 -DKW=8 -DKLP=16 -DKMF=1 -DGPSIG_FO_LB=2
wait
ls tools/bin
