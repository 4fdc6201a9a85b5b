#!/bin/bash
# stride-2 halo wgrad on the shared route: GPU suites touching conv routing (both engines), benches, kernel table
TAG=${1:-ws2b}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/ws2b_$TAG.log; : > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_geometry.py tests/test_gpu_model.py tests/test_cpp_host_blocks.py tests/test_cpp_host_api.py tests/test_conv_routing.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $L 2>&1 || exit $?
  timeout -k 10 200 python bench.py --steps 40 --warmup 8 --engine python >> $L 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --model resnet50_tiny_imagenet --batch 256 >> $L 2>&1 || exit $?
bash tools/gpu_prof.sh r18_$TAG --steps 15 --warmup 5
