#!/bin/bash
# Kernel experiment: conv/GEMM kernel numerics, then per env setting a per-shape conv bench and a
# headline bench. usage (via gpurun): bash tools/gpu_exp.sh TAG "SHAPES|all" "ENV_1" "ENV_2" ...
# each ENV_i is a space-separated list of VAR=value (X=0 for "defaults"); results are appended to
# gpurun_out/exp_TAG.txt
TAG=${1:-exp}; SH=${2:-all}; shift 2
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || exit $?
SARG=""; [ "$SH" != "all" ] && SARG="--shapes $SH"
O=gpurun_out/exp_$TAG.txt; : > $O
i=0
for E in "$@"; do
  echo "=== $E" >> $O
  env $E timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 $SARG > gpurun_out/c_${TAG}_$i.log 2>&1 || exit $?
  cat gpurun_out/c_${TAG}_$i.log >> $O
  env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_${TAG}_$i.log 2>&1 || exit $?
  grep '^{' gpurun_out/b_${TAG}_$i.log | cut -c1-200 >> $O
  i=$((i+1))
done
