#!/bin/bash
# g2 3-stage pipeline: numerics, per-shape A/B vs 2-stage, end-to-end bench; new generic/tensor-op tests
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_tensor_ops.py -x -q -m gpu > gpurun_out/t9.log 2>&1 || exit $?
DCNN_G2_STAGES=2 timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only fwd > gpurun_out/c9_2.log 2>&1 || exit $?
DCNN_G2_STAGES=3 timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 > gpurun_out/c9_3.log 2>&1 || exit $?
DCNN_G2_STAGES=2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b9.log 2>&1 || exit $?
DCNN_G2_STAGES=3 timeout -k 10 300 python bench.py --steps 30 --warmup 5 >> gpurun_out/b9.log 2>&1
