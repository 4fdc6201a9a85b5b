#!/bin/bash
# C++ data parallelism + the RCCL core refactor: the RCCL / DP GPU tests (Python wrapper), the C++
# host GPU tests (world-1 DP among them), the C++ trainer with --dp at world 1 vs without.
# usage (via gpurun): bash tools/gpu_cpp_dp.sh TAG
TAG=${1:-dp}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/cppdp_$TAG.log; : > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dp.py tests/test_cpp_host_blocks.py -m gpu -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch 256 --steps 40 --bench >> $L 2>&1 || exit $?
RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch 256 --steps 40 --bench --dp >> $L 2>&1 || exit $?
