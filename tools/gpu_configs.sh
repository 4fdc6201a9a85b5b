#!/bin/bash
# Measure the non-headline BASELINE.json configs on one MI355X:
# ResNet-9 CIFAR-10 fp32 (+bf16), ResNet-18 fp32, ResNet-50 Tiny-ImageNet bf16 (single GPU), and
# the ResNet-50 pipeline schedules (in-process coordinator; every stage on cuda:0 on the one-GPU box).
# usage (via gpurun): bash tools/gpu_configs.sh TAG
TAG=${1:-cfg}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/configs_$TAG.jsonl; : > $O
E=gpurun_out/configs_$TAG.err; : > $E
run() { echo "== $*" >> $E; timeout -k 10 240 "$@" > gpurun_out/cur.out 2>>$E; rc=$?; grep '^{' gpurun_out/cur.out >> $O; return $rc; }
run python bench.py --model resnet9_cifar10 --dtype fp32 --batch 128 --steps 30 --warmup 5 || exit $?
run python bench.py --model resnet9_cifar10 --dtype fp32 --batch 256 --steps 30 --warmup 5 || exit $?
run python bench.py --model resnet9_cifar10 --dtype fp32 --f32-mode exact --batch 128 --steps 30 --warmup 5 || exit $?
run python bench.py --model resnet18_tiny_imagenet --dtype fp32 --f32-mode exact --batch 256 --steps 20 --warmup 5 || exit $?
run python bench.py --model resnet9_cifar10 --dtype bf16 --batch 256 --steps 30 --warmup 5 || exit $?
run python bench.py --model resnet18_tiny_imagenet --dtype fp32 --batch 256 --steps 20 --warmup 5 || exit $?
run python bench.py --model resnet50_tiny_imagenet --dtype bf16 --batch 256 --steps 20 --warmup 5 || exit $?
run python benchmarks/pipeline_bench.py --stages 1 --schedule sync --steps 10 --warmup 3 || exit $?
run python benchmarks/pipeline_bench.py --stages 4 --schedule sync --steps 10 --warmup 3 || exit $?
run python benchmarks/pipeline_bench.py --stages 4 --schedule semi_async --steps 10 --warmup 3 || exit $?
run python benchmarks/pipeline_bench.py --stages 8 --schedule semi_async --steps 10 --warmup 3 || exit $?
run python bench.py --batch 512 --steps 20 --warmup 5 || exit $?
run python bench.py --batch 1024 --steps 20 --warmup 5 || exit $?
run python bench.py --pg --steps 30 --warmup 5 || exit $?
run python bench.py --batch 128 --steps 30 --warmup 5 || exit $?
run python bench.py --batch 64 --steps 30 --warmup 5 || exit $?
run python bench.py --model resnet50_tiny_imagenet --dtype bf16 --batch 32 --steps 30 --warmup 5 || exit $?
run python benchmarks/pipeline_bench.py --stages 4 --schedule 1f1b --steps 10 --warmup 3 || exit $?
run python benchmarks/pipeline_bench.py --stages 8 --schedule sync --steps 10 --warmup 3 || exit $?
run python bench.py --engine native --steps 30 --warmup 5 || exit $?
run python bench.py --engine native --batch 64 --steps 30 --warmup 5 || exit $?
run python bench.py --steps 30 --warmup 5 || exit $?
echo "== native pipeline" >> $E
timeout -k 10 300 dcnn_amd/bin/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 --transport ipc --partitioner flops > gpurun_out/cur.out 2>>$E || exit $?
grep '^{' gpurun_out/cur.out >> $O
timeout -k 10 300 dcnn_amd/bin/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule sync --steps 8 --bench 2 --transport ipc --partitioner flops > gpurun_out/cur.out 2>>$E || exit $?
grep '^{' gpurun_out/cur.out >> $O
run python benchmarks/loader_bench.py --images-per-class 50 --batch 256 --steps 40 || exit $?
