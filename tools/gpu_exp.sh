#!/bin/bash
# Kernel experiment: numerics of the conv/GEMM kernels, per-shape conv bench (A/B via env), bench.
# usage (via gpurun): bash tools/gpu_exp.sh TAG "ENV_A" "ENV_B"
TAG=${1:-exp}; A=${2:-X=0}; B=${3:-X=1}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || exit $?
env $A timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 > gpurun_out/c_${TAG}_a.log 2>&1 || exit $?
env $B timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 > gpurun_out/c_${TAG}_b.log 2>&1 || exit $?
env $A timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_${TAG}_a.log 2>&1 || exit $?
env $B timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_${TAG}_b.log 2>&1
