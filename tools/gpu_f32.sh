#!/bin/bash
# fp32 configs: dcnn_amd fp32 benches + kernel profiles, PyTorch fp32 baselines for the same models.
TAG=${1:-f32}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/f32_$TAG.jsonl; : > $O
timeout -k 10 200 python bench.py --dtype fp32 --steps 20 --warmup 3 2>>gpurun_out/f32_$TAG.err | grep '^{' >> $O || exit $?
timeout -k 10 200 python bench.py --model resnet9_cifar10 --dtype fp32 --batch 128 --steps 20 --warmup 3 2>>gpurun_out/f32_$TAG.err | grep '^{' >> $O || exit $?
timeout -k 10 300 python benchmarks/torch_baseline.py --model resnet9_cifar10 --mode fp32 --batch 128 --steps 20 --warmup 5 2>>gpurun_out/f32_$TAG.err | grep '^{' >> $O || exit $?
timeout -k 10 300 python benchmarks/torch_baseline.py --model resnet9_cifar10 --mode bf16 --batch 128 --steps 20 --warmup 5 2>>gpurun_out/f32_$TAG.err | grep '^{' >> $O || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_f32_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dtype fp32 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_f32_$TAG.log 2>&1
