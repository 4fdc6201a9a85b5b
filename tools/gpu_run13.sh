#!/bin/bash
# hconv taps-per-step A/B (1 vs 3) + numerics
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "conv or teacher or graph" > gpurun_out/t13.log 2>&1 || exit $?
DCNN_HCONV_TPS=1 timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only fwd > gpurun_out/c13_1.log 2>&1 || exit $?
DCNN_HCONV_TPS=3 timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only fwd > gpurun_out/c13_3.log 2>&1 || exit $?
DCNN_HCONV_TPS=3 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b13.log 2>&1
