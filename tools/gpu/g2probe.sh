#!/bin/bash
# strided dgrad (gemm_g2 grouped phases) with the production backward-BN epilogue: variants
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/g2probe.log; : > $L
S=l2.b1c1,l3.b1c1,l4.b1c1,l2.proj
run() { echo "== $*" >> $L; timeout -k 10 120 python benchmarks/conv_bench.py --only dgrad --shapes $S --iters 20 "$@" >> $L 2>&1 || exit 1; }
run
run --bnb
run --bnb --no-group
DCNN_G2_STAGES=2 run --bnb
DCNN_G2_TILE=64x64 run --bnb
DCNN_G2_TILE=128x128 run --bnb
DCNN_G2_TILE=64x128 run --bnb
cat $L
