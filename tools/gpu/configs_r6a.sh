#!/bin/bash
# round-6 BASELINE config sweep, part a (tools/gpu_configs.sh split in two calls)
TAG=${1:-r6}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/configs_$TAG.jsonl; E=gpurun_out/configs_$TAG.err
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
