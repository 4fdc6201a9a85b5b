#!/bin/bash
# halo wgrad: numerics, conv bench (256 / 512 target workgroups), bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t15.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only wgrad > gpurun_out/c15.log 2>&1 || exit $?
DCNN_HWGRAD_BLOCKS=512 timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only wgrad > gpurun_out/c15b.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b15.log 2>&1 || exit $?
