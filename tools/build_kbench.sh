#!/bin/bash
# Build the kbench A/B variants (tools/kbench.hip) into tools/bin/.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize"
b() { name=$1; shift; hipcc $F -DVARIANT=\"$name\" "$@" tools/kbench.hip -o tools/bin/$name & }
b base_plain -DGPSIG_FO_BLOCKED=0 -DGPSIG_D2_RECUR=0
b blocked_exact -DGPSIG_FO_BLOCKED=1 -DGPSIG_D2_RECUR=0
b blocked_recur -DGPSIG_FO_BLOCKED=1 -DGPSIG_D2_RECUR=1
b plain_recur -DGPSIG_FO_BLOCKED=0 -DGPSIG_D2_RECUR=1
b blocked_exact_lb2 -DGPSIG_FO_BLOCKED=1 -DGPSIG_D2_RECUR=0 -DGPSIG_FO_LB=2
wait
ls tools/bin
