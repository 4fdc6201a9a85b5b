#!/bin/bash
# Kernel iteration: the given GPU test files, per-shape conv_bench (ResNet-18 and -50 sets), benches.
# usage (via gpurun): bash tools/gpu_iter.sh TAG test_file...
TAG=${1:-it}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --set r50 > gpurun_out/cb_${TAG}_r50.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l2.proj,l3.proj > gpurun_out/cb_${TAG}_r18.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --model resnet50_tiny_imagenet --steps 20 --warmup 5 > gpurun_out/b50_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --model resnet50_tiny_imagenet --batch 32 --steps 30 --warmup 5 > gpurun_out/b50s_$TAG.log 2>&1 || exit $?
