#!/bin/bash
# round-6 BASELINE config sweep, part b (tools/gpu_configs.sh split in two calls)
TAG=${1:-r6}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/configs_$TAG.jsonl; E=gpurun_out/configs_$TAG.err
run() { echo "== $*" >> $E; timeout -k 10 240 "$@" > gpurun_out/cur.out 2>>$E; rc=$?; grep '^{' gpurun_out/cur.out >> $O; return $rc; }
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
