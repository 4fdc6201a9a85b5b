#!/bin/bash
# round-6 kernel tables (C++ engine: ResNet-18 b256, ResNet-50 b32) + BN bandwidth tables with the copy reference
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet18 --batch 256 > gpurun_out/bn_bw_r18.md 2>&1 || { tail -20 gpurun_out/bn_bw_r18.md; exit 1; }
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet50 --batch 256 > gpurun_out/bn_bw_r50.md 2>&1 || { tail -20 gpurun_out/bn_bw_r50.md; exit 1; }
bash tools/gpu_prof_cpp.sh r18_r6 --model resnet18_tiny_imagenet --batch 256 --steps 20 --warmup 5 --loss softmax_ce --bench || exit 1
bash tools/gpu_prof_cpp.sh r50b32_r6 --model resnet50_tiny_imagenet --batch 32 --steps 20 --warmup 5 --loss softmax_ce --bench || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu > gpurun_out/t_bn.log 2>&1 || { tail -30 gpurun_out/t_bn.log; exit 1; }
tail -2 gpurun_out/t_bn.log
head -30 gpurun_out/prof_r18_r6.md; head -30 gpurun_out/prof_r50b32_r6.md; grep -h "copy\|mean_pct" gpurun_out/bn_bw_r18.md gpurun_out/bn_bw_r50.md
