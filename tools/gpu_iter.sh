#!/bin/bash
# One iteration: kernel GPU tests, conv shapes, hconv3 timeline, ResNet-18 + ResNet-50 benches.
# usage (via gpurun): bash tools/gpu_iter.sh TAG
TAG=${1:-it}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_hconv3.py tests/test_gpu_kernels.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l1.c,l2.c,l3.c,l4.c --v3 1 > gpurun_out/cb_$TAG.log 2>&1 || exit $?
timeout -k 10 120 python benchmarks/hconv3_timeline.py --batch 256 --shapes l1.c,l2.c > gpurun_out/tl_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --model resnet50_tiny_imagenet --steps 20 --warmup 5 > gpurun_out/b50_$TAG.log 2>&1 || exit $?
