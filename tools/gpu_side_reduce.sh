#!/bin/bash
# A/B of the mid-backward side-stream split-K reduce (DCNN_SIDE_REDUCE_MB) on ResNet-18 b256 /
# b64 and ResNet-50 b256, interleaved; final loss printed for the bit-identity check.
# usage (via gpurun): bash tools/gpu_side_reduce.sh TAG
TAG=${1:-side}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/side_$TAG.log; : > $L
for rep in 1 2; do
  for MB in 0 64 160; do
    echo "== MB=$MB rep=$rep" >> $L
    DCNN_SIDE_REDUCE_MB=$MB timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $L 2>&1 || exit $?
    DCNN_SIDE_REDUCE_MB=$MB timeout -k 10 200 python bench.py --batch 64 --steps 40 --warmup 8 >> $L 2>&1 || exit $?
    DCNN_SIDE_REDUCE_MB=$MB timeout -k 10 200 python bench.py --model resnet50_tiny_imagenet --steps 20 --warmup 5 >> $L 2>&1 || exit $?
  done
done
