#!/bin/bash
# ResNet-50 K >= 1024 1x1 convs: halo kernel vs the routing table's GEMM choice vs torch.mm (hipBLASLt)
TAG=${1:-1x1}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/c1x1_$TAG.log; : > $L
for B in 32 256; do
  echo "== batch $B halo-1x1 on (+ torch.mm)" >> $L
  timeout -k 10 200 python benchmarks/conv_bench.py --set r50 --batch $B --iters 20 --shapes r1.c1,r2.c1,r2.c3,r3.c1,r3.c3,r4.c1,r4.c3 --torch-mm >> $L 2>&1 || exit $?
  echo "== batch $B halo-1x1 off" >> $L
  timeout -k 10 200 python benchmarks/conv_bench.py --set r50 --batch $B --iters 20 --shapes r3.c1,r3.c3,r4.c1,r4.c3 --halo-1x1 0 >> $L 2>&1 || exit $?
done
