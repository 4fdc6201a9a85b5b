#!/bin/bash
# full GPU suite, conv / step benches, C++ trainer vs eager, exact-fp32 configs + profile, in one
# call; stops at the first GPU fault / abort / time limit.  usage: bash tools/gpu_cf.sh TAG
TAG=${1:-cf}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ok() { case $1 in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log; ok $rc || exit $rc
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l1.c,l2.c,l3.c,l4.c > gpurun_out/cb_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 64 --iters 20 --shapes l1.c,l2.c,l3.c,l4.c >> gpurun_out/cb_$TAG.log 2>&1 || exit $?
L=gpurun_out/b_$TAG.log; : > $L
for B in 256 64; do
  timeout -k 10 240 python bench.py --batch $B --steps 30 --warmup 5 >> $L 2>&1 || exit $?
  timeout -k 10 240 python bench.py --batch $B --graph 0 --steps 20 --warmup 3 >> $L 2>&1 || exit $?
  timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch $B --steps 20 --bench >> $L 2>&1 || exit $?
done
timeout -k 10 300 dcnn_amd/bin/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 >> $L 2>&1 || exit $?
timeout -k 10 240 python bench.py --model resnet9_cifar10 --dtype fp32 --f32-mode exact --batch 128 --steps 30 --warmup 5 >> $L 2>&1 || exit $?
timeout -k 10 240 python bench.py --model resnet18_tiny_imagenet --dtype fp32 --f32-mode exact --batch 256 --steps 20 --warmup 5 >> $L 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_f32$TAG -o run -- python3 $R/bench.py --model resnet9_cifar10 --dtype fp32 --f32-mode exact --batch 128 --steps 10 --warmup 3 > $R/gpurun_out/prof_f32$TAG.log 2>&1 || exit $?
cd $R && DB=$(find gpurun_out/prof_f32$TAG -name 'run_results.db' -print -quit) && python tools/prof_summary.py $DB > gpurun_out/prof_f32$TAG.md 2>&1
exit 0
