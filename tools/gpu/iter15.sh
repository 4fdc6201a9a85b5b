#!/bin/bash
# BN vectors-per-lane sweep on the large passes: microbench + end-to-end (R18 b256 / b128, R50 b32)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/it15.log; : > $L
for U in 1 2 4; do
  echo "== DCNN_BN_U=$U" >> $L
  DCNN_BN_U=$U timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet18 --batch 256 >> $L 2>&1 || exit 1
done
bash tools/gpu/perf_ab.sh bnu DCNN_BN_U=1 DCNN_BN_U=2 DCNN_BN_U=4 >> $L 2>&1 || exit 1
AB_BATCH=128 bash tools/gpu/perf_ab.sh bnu128 DCNN_BN_U=1 DCNN_BN_U=4 >> $L 2>&1 || exit 1
grep -E "^==|l1 |l2 |bnu" $L | grep -v copy
