#!/bin/bash
# g1s store-path experiments (DCNN_G1S_DBG): tests on the given paths, then per-shape times.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-g1dbg}; shift
for D in "$@"; do
  DCNN_G1S_DBG=$D timeout -k 10 200 python -u -m pytest tests/test_gpu_g1s.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_${TAG}_$D.log 2>&1 || exit $?
done
for D in "$@"; do
  echo "== dbg $D" >> gpurun_out/cb_$TAG.log
  DCNN_G1S_DBG=$D timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --set r50 --shapes r1.c1a,r1.c3,r2.c3,r1.c1,r2.c1 >> gpurun_out/cb_$TAG.log 2>&1 || exit $?
done
