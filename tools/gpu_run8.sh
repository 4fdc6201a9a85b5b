#!/bin/bash
# fp32 path tests + fp32 ResNet-9 CIFAR bench + bf16 regression bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "fp32" > gpurun_out/t8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model resnet9_cifar10 --dtype fp32 --batch 256 --steps 20 --warmup 5 > gpurun_out/b8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model resnet9_cifar10 --dtype bf16 --batch 256 --steps 20 --warmup 5 >> gpurun_out/b8.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> gpurun_out/b8.log 2>&1
