#!/bin/bash
# Round 6 forward A/B (tools/kbench.hip): scalar record loads (GPSIG_SREC) and the scans issued before the
# row's cells (GPSIG_SCAN_FIRST 1: prefixes kept live, 2: recomputed) at C2 (W10/LP10), H (W8/LP16) and C5.
# (Both switches were removed from the sources after this A/B -- gpurun_out/r6h, DESIGN.md 2.1: -0.4 % and 2x
#  slower -- so rebuilding these variants now gives four copies of the kept kernel.)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize"
b() { name=$1; shift; /opt/rocm/bin/hipcc $F -DVARIANT=\"$name\" "$@" tools/kbench.hip -o tools/bin/$name & }
C2="-DKL=100 -DKW=10 -DKLP=10"
H="-DKL=128 -DKW=8 -DKLP=16"
C5="-DKL=128 -DKW=8 -DKLP=16 -DKD=8 -DKM=6"
b c2_base $C2
b c2_srec $C2 -DGPSIG_SREC=1
b c2_sf1 $C2 -DGPSIG_SREC=1 -DGPSIG_SCAN_FIRST=1
b c2_sf2 $C2 -DGPSIG_SREC=1 -DGPSIG_SCAN_FIRST=2
wait
b h_base $H
b h_sf1 $H -DGPSIG_SREC=1 -DGPSIG_SCAN_FIRST=1
b h_sf2 $H -DGPSIG_SREC=1 -DGPSIG_SCAN_FIRST=2
b c5_base $C5
wait
b c5_sf1 $C5 -DGPSIG_SREC=1 -DGPSIG_SCAN_FIRST=1
b c5_sf2 $C5 -DGPSIG_SREC=1 -DGPSIG_SCAN_FIRST=2
wait
