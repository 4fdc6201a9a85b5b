#!/bin/bash
# hconv3 epilogue ablations (DCNN_HCONV3_DBG bits: 1 no output stores, 2 no statistics)
TAG=${1:-dbg}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for D in 0 1 2 3; do
  echo "== dbg $D" >> gpurun_out/dbg_$TAG.log
  DCNN_HCONV3_DBG=$D timeout -k 10 120 python benchmarks/hconv3_timeline.py --batch 256 --shapes l1.c,l2.c >> gpurun_out/dbg_$TAG.log 2>&1 || exit $?
  DCNN_HCONV3_DBG=$D timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l1.c,l2.c --only fwd >> gpurun_out/dbg_$TAG.log 2>&1 || exit $?
done
