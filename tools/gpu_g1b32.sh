#!/bin/bash
# g1s vs gathered GEMM per shape at small batches (ResNet-50 1x1 shapes)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for B in 32 64; do
for E in 1 0; do
  echo "== batch $B DCNN_G1S=$E" >> gpurun_out/cb_g1b32.log
  DCNN_G1S=$E timeout -k 10 200 python benchmarks/conv_bench.py --batch $B --iters 20 --set r50 --shapes r1.c1a,r1.c1,r1.c3,r2.c1,r2.c3,r2.proj,r3.c1,r3.c3,r4.c3 --only fwd >> gpurun_out/cb_g1b32.log 2>&1 || exit $?
  DCNN_G1S=$E timeout -k 10 200 python benchmarks/conv_bench.py --batch $B --iters 20 --set r50 --shapes r1.c1a,r1.c1,r1.c3,r2.c1,r2.c3,r3.c1,r3.c3,r4.c1 --only dgrad >> gpurun_out/cb_g1b32.log 2>&1 || exit $?
done
done
