#!/bin/bash
# Conv kernel iteration: hconv3 GPU tests, per-shape conv_bench (hconv3 on / off), headline bench.
# usage (via gpurun): bash tools/gpu_conv.sh TAG [batch]
TAG=${1:-conv}; B=${2:-256}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hconv3.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch $B --iters 20 --shapes l1.c,l2.c,l3.c,l4.c --v3 1 > gpurun_out/cb_${TAG}_v3.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch $B --iters 20 --shapes l1.c,l2.c,l3.c,l4.c --v3 0 > gpurun_out/cb_${TAG}_v2.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --batch 64 --steps 30 --warmup 5 > gpurun_out/b64_$TAG.log 2>&1 || exit $?
