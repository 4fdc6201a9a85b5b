#!/bin/bash
# wide-C BatchNorm launch shape sweep (ResNet-50 b256 shapes)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/it11.log; : > $L
for W in 0 1 2 0 1 2; do
  echo "== DCNN_BN_WIDE=$W" >> $L
  DCNN_BN_WIDE=$W timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet50 --batch 256 >> $L 2>&1 || { tail -20 $L; exit 1; }
done
grep -E "^==|l3.w|l4.w|mean_pct" $L | grep -v dual
