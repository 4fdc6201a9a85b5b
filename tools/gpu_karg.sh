#!/bin/bash
# kernel-argument prefetch A/B: hconv3 phase timeline + conv bench + the headline bench
TAG=${1:-karg}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/karg_$TAG.log; : > $L
timeout -k 10 150 python benchmarks/hconv3_timeline.py --shapes l1.c,l2.c,l3.c >> $L 2>&1 || exit $?
timeout -k 10 150 python benchmarks/hconv3_timeline.py --op dgrad --shapes l1.c,l2.c >> $L 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $L 2>&1 || exit $?
  timeout -k 10 200 python bench.py --batch 64 --steps 40 --warmup 8 >> $L 2>&1 || exit $?
  timeout -k 10 200 python bench.py --model resnet50_tiny_imagenet --batch 32 --steps 30 --warmup 8 >> $L 2>&1 || exit $?
done
