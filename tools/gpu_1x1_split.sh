#!/bin/bash
# ResNet-50 b32 K >= 1024 1x1 convs on the halo kernel: split-K target / least work per split sweep
TAG=${1:-split}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/c1x1s_$TAG.log; : > $L
for T in 256 512 1024; do for MW in 1 2 4 8; do
  echo "== target $T min_work $MW" >> $L
  timeout -k 10 120 python benchmarks/conv_bench.py --set r50 --batch 32 --iters 20 --shapes r3.c1,r3.c3,r4.c1,r4.c3 --split-target $T --split-min-work $MW >> $L 2>&1 || exit $?
done; done
