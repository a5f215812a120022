#!/bin/bash
# Build the Gram-VJP A/B variants (tools/kbench_vjp.hip) into tools/bin/: the round-5 kernel (sig_bwd.h) and the
# packed column-pair kernel (sig_bwd_pk.h), with the training step's saved state (KSTATE=1), D = 5, M = 5:
# L = 100 (C2: round-5 LP = 20 x W = 5 vs packed LP = 32 x W = 4), L = 64 (both LP = 16 x W = 4), L = 128
# (both LP = 32 x W = 4).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/bin
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -mllvm -amdgpu-atomic-optimizer-strategy=None"
b() { name=$1; shift; /opt/rocm/bin/hipcc $F -DVARIANT=\"$name\" "$@" tools/kbench_vjp.hip -o tools/bin/$name & }
b v_r5_st -DKW=5 -DKLP=20 -DKSTATE=1
b v_pk4_st -DKW=4 -DKLP=32 -DKPK=1 -DKSTATE=1
b v_r5_l64 -DKL=64 -DKW=4 -DKLP=16 -DKSTATE=1
b v_pk_l64 -DKL=64 -DKW=4 -DKLP=16 -DKPK=1 -DKSTATE=1
b v_r5_l128 -DKL=128 -DKW=4 -DKLP=32 -DKSTATE=1
b v_pk_l128 -DKL=128 -DKW=4 -DKLP=32 -DKPK=1 -DKSTATE=1
wait
ls tools/bin
