#!/bin/bash
# BN apply passes: LDS tables vs per-lane register coefficients, grid caps; BN GPU tests
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/it9.log; : > $L
for M in resnet18 resnet50; do
  for V in "0 1024" "1 1024" "1 2048" "1 512"; do
    set -- $V
    echo "== $M DCNN_BN_REG=$1 DCNN_BN_GRID_CAP=$2" >> $L
    DCNN_BN_REG=$1 DCNN_BN_GRID_CAP=$2 timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model $M --batch 256 >> $L 2>&1 || { tail -20 $L; exit 1; }
  done
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
grep -E "^==|mean_pct|passed|failed" $L
