#!/bin/bash
# Round-end check: full GPU suite, smoke, default bench, and refreshed kernel tables for
# ResNet-18 b256 and ResNet-50 b32 / b256. Stops at the first failure.
# usage (via gpurun): bash tools/gpu_final.sh TAG
TAG=${1:-final}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ok() { case $1 in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
for B in 32 256; do
  timeout -k 10 300 python bench.py --model resnet50_tiny_imagenet --batch $B >> gpurun_out/bench_$TAG.log 2>&1 || exit $?
done
bash tools/gpu_prof.sh r18_$TAG --steps 15 --warmup 5 || exit $?
bash tools/gpu_prof.sh r50b32_$TAG --model resnet50_tiny_imagenet --batch 32 --steps 15 --warmup 5 || exit $?
bash tools/gpu_prof.sh r50b256_$TAG --model resnet50_tiny_imagenet --batch 256 --steps 15 --warmup 5
