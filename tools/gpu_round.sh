#!/bin/bash
# End-of-round GPU pass: full GPU suite, smoke, the default bench, the BASELINE.json config sweep
# (tools/gpu_configs.sh), the C++ trainer and the all-native pipeline. Stops at the first GPU
# fault / abort / time limit.  usage (via gpurun): bash tools/gpu_round.sh TAG
TAG=${1:-round}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ok() { case $1 in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit $?
bash tools/gpu_configs.sh $TAG || exit $?
L=gpurun_out/cpp_$TAG.log; : > $L
for B in 256 64; do
  timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch $B --steps 30 --bench >> $L 2>&1 || exit $?
  timeout -k 10 240 python bench.py --batch $B --graph 0 --steps 30 --warmup 5 >> $L 2>&1 || exit $?
done
timeout -k 10 300 dcnn_amd/bin/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 >> $L 2>&1
