#!/bin/bash
# Round 6 forward A/B (tools/kbench.hip): the range check on the first column pair only (GPSIG_P0CHECK) at C2, H and C5.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize"
b() { name=$1; shift; /opt/rocm/bin/hipcc $F -DVARIANT=\"$name\" "$@" tools/kbench.hip -o tools/bin/$name & }
C2="-DKL=100 -DKW=10 -DKLP=10"
H="-DKL=128 -DKW=8 -DKLP=16"
C5="-DKL=128 -DKW=8 -DKLP=16 -DKD=8 -DKM=6"
b c2_base $C2 -DGPSIG_P0CHECK=0
b c2_plo $C2
b h_base $H -DGPSIG_P0CHECK=0
b h_plo $H
wait
b c5_base $C5 -DGPSIG_P0CHECK=0
b c5_plo $C5
wait
