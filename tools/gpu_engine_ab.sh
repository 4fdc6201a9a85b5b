#!/bin/bash
# C++ vs Python engine on the bench.py configs (auto = C++ on one GPU)
TAG=${1:-eng}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/engine_$TAG.log; : > $L
for M in "resnet18_tiny_imagenet 256" "resnet18_tiny_imagenet 64" "resnet50_tiny_imagenet 256" "resnet50_tiny_imagenet 32" "resnet18_tiny_imagenet 1024"; do
  set -- $M
  for E in auto python; do
    echo "== $1 $2 $E" >> $L
    timeout -k 10 240 python bench.py --model $1 --batch $2 --engine $E --steps 30 --warmup 8 >> $L 2>&1 || exit $?
  done
done
