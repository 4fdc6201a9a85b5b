#!/bin/bash
# BatchNorm apply-pass launch-shape sweep: bash tools/gpu_bnsweep.sh TAG "ENV_1" "ENV_2" ...
TAG=${1:-bns}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/bnsweep_$TAG.txt; : > $O
for E in "$@"; do
  echo "== $E" >> $O
  env $E timeout -k 10 200 python benchmarks/bn_bench.py --batch 256 >> $O 2>/dev/null || exit $?
done
