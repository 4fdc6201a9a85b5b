#!/bin/bash
# g1s variants: tests under each env setting, then per-shape times (ResNet-50 1x1 shapes).
# usage (via gpurun): bash tools/gpu_g1dbg.sh TAG "ENV=V ..." ...   ("-" = defaults)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-g1dbg}; shift
n=0
for E in "$@"; do
  [ "$E" = "-" ] && E=""
  n=$((n+1))
  env $E timeout -k 10 200 python -u -m pytest tests/test_gpu_g1s.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_${TAG}_$n.log 2>&1 || exit $?
  echo "== $E" >> gpurun_out/cb_$TAG.log
  env $E timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --set r50 --shapes r1.c1a,r1.c3,r2.c3,r1.c1,r2.c1 >> gpurun_out/cb_$TAG.log 2>&1 || exit $?
done
