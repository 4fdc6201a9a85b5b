#!/bin/bash
# halo conv: numerics then per-shape A/B and end-to-end bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -k "conv" > gpurun_out/t12.log 2>&1 || exit $?
timeout -k 10 600 python -m pytest tests/test_gpu_model.py -x -q > gpurun_out/t12m.log 2>&1 || exit $?
DCNN_HCONV=0 timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only fwd > gpurun_out/c12_0.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 > gpurun_out/c12_1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b12.log 2>&1
