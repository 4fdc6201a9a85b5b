#!/bin/bash
# hconv3 iteration: GPU tests of the kernel, conv_bench (ResNet-18 3x3 shapes at batch 256 and 64),
# timeline, benches.  usage (via gpurun): bash tools/gpu_h3.sh TAG
TAG=${1:-h3}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hconv3.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l1.b1c1,l1.c,l2.c,l3.c,l4.c > gpurun_out/cb_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 64 --iters 20 --shapes l1.c,l2.c,l3.c,l4.c >> gpurun_out/cb_$TAG.log 2>&1 || exit $?
timeout -k 10 120 python benchmarks/hconv3_timeline.py --batch 256 --shapes l1.c,l2.c,l3.c,l4.c > gpurun_out/tl_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --batch 64 --steps 30 --warmup 5 > gpurun_out/b64_$TAG.log 2>&1 || exit $?
