#!/bin/bash
# C++ host API on the GPU: native pipeline stages test, C++ ResNet-18 trainer throughput vs the
# Python front end's eager step at the same batch.  usage (via gpurun): bash tools/gpu_cpp.sh TAG
TAG=${1:-cpp}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/cpp_$TAG.log; : > $L
timeout -k 10 300 python -u -m pytest tests/test_native_pipeline.py tests/test_cpp_host_blocks.py -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for B in 64 256; do
  timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch $B --steps 20 --bench >> $L 2>&1 || exit $?
  timeout -k 10 240 python bench.py --batch $B --graph 0 --steps 20 --warmup 3 >> $L 2>&1 || exit $?
done
