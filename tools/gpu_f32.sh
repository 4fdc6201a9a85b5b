#!/bin/bash
# exact-fp32 path: GPU tests of the fp32 kernels, the fp32 BASELINE configs, a kernel profile.
# usage (via gpurun): bash tools/gpu_f32.sh TAG
TAG=${1:-f32}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=gpurun_out/f32_$TAG.log; : > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_im2col.py -m gpu -q -rf -k "f32 or fp32 or float32 or im2col" --timeout 240 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
timeout -k 10 240 python bench.py --model resnet9_cifar10 --dtype fp32 --f32-mode exact --batch 128 --steps 30 --warmup 5 >> $L 2>&1 || exit $?
timeout -k 10 240 python bench.py --model resnet18_tiny_imagenet --dtype fp32 --f32-mode exact --batch 256 --steps 20 --warmup 5 >> $L 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --model resnet9_cifar10 --dtype fp32 --f32-mode exact --batch 128 --steps 10 --warmup 3 > $R/gpurun_out/prof_$TAG.log 2>&1 || exit $?
cd $R && DB=$(find gpurun_out/prof_$TAG -name 'run_results.db' -print -quit) && python tools/prof_summary.py $DB > gpurun_out/prof_$TAG.md 2>&1 || exit $?
bash tools/gpu_pmc_f32.sh ${TAG}p
