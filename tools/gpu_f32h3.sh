#!/bin/bash
# Exact fp32 on the persistent halo conv / halo wgrad: the fp32 kernel tests, the fp32 model tests,
# then ResNet-9 b128 / ResNet-18 b256 exact fp32 with the halo kernels on (default) and with the
# fp32 halo wgrad off, and a kernel table of ResNet-9 exact.
# usage (via gpurun): bash tools/gpu_f32h3.sh TAG
TAG=${1:-f32}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/f32h3_$TAG.log; : > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "fp32" -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_im2col.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for HW in 1 0; do
  echo "== DCNN_HW_F32=$HW" >> $L
  DCNN_HW_F32=$HW timeout -k 10 200 python bench.py --model resnet9_cifar10 --dtype fp32 --f32-mode exact --batch 128 --steps 30 --warmup 5 >> $L 2>&1 || exit $?
  DCNN_HW_F32=$HW timeout -k 10 200 python bench.py --model resnet18_tiny_imagenet --dtype fp32 --f32-mode exact --batch 256 --steps 20 --warmup 5 >> $L 2>&1 || exit $?
done
bash tools/gpu_prof.sh r9f32_$TAG --model resnet9_cifar10 --dtype fp32 --f32-mode exact --batch 128 --steps 15 --warmup 5
