#!/bin/bash
# Per-shape conv data: ResNet-18 shapes (hconv3 on / off), ResNet-50 shapes, hconv3 epilogue ablations.
# usage (via gpurun): bash tools/gpu_convdata.sh TAG
TAG=${1:-cd}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --v3 1 > gpurun_out/cb_${TAG}_r18.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --v3 0 --shapes l1.c,l2.c > gpurun_out/cb_${TAG}_r18v2.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --set r50 > gpurun_out/cb_${TAG}_r50.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 32 --iters 20 --set r50 > gpurun_out/cb_${TAG}_r50b32.log 2>&1 || exit $?
bash tools/gpu_h3dbg.sh $TAG
