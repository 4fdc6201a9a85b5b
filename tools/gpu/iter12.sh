#!/bin/bash
# ResNet-50 K >= 1024 1x1 convs: gemm_g2 split-K (default) vs without vs torch.mm (hipBLASLt)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/it12.log; : > $L
for B in 32 256; do
  echo "== batch $B split-K on (+ torch.mm)" >> $L
  timeout -k 10 200 python benchmarks/conv_bench.py --set r50 --batch $B --iters 20 --shapes r3.c1,r3.c3,r4.c1,r4.c3 --torch-mm >> $L 2>&1 || exit 1
  echo "== batch $B split-K off" >> $L
  DCNN_G2_SPLITK=0 timeout -k 10 200 python benchmarks/conv_bench.py --set r50 --batch $B --iters 20 --shapes r3.c1,r3.c3,r4.c1,r4.c3 >> $L 2>&1 || exit 1
done
cat $L | grep -v amdgpu.ids
