#!/bin/bash
# fp32 split-precision check: fp32 kernel tests (both modes), fp32 model tests, fp32 benches (split and exact).
TAG=${1:-f32b}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -rf -k "fp32 or f32 or float32" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
case $rc in 0|1|5) ;; *) exit $rc ;; esac
O=gpurun_out/f32_$TAG.jsonl; : > $O
timeout -k 10 200 python bench.py --dtype fp32 --steps 20 --warmup 3 2>>gpurun_out/f32_$TAG.err | grep '^{' >> $O || exit $?
timeout -k 10 200 python bench.py --model resnet9_cifar10 --dtype fp32 --batch 128 --steps 20 --warmup 3 2>>gpurun_out/f32_$TAG.err | grep '^{' >> $O || exit $?
DCNN_F32_EXACT=1 timeout -k 10 200 python bench.py --model resnet9_cifar10 --dtype fp32 --batch 128 --steps 20 --warmup 3 2>>gpurun_out/f32_$TAG.err | grep '^{' >> $O || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
