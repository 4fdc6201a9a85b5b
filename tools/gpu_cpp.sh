#!/bin/bash
# C++ host API on the GPU: native pipeline / host API GPU tests, the C++ ResNet-18 trainer's
# throughput (vs the Python front end's eager step: run bench.py --graph 0 separately), the
# all-native 4-stage pipeline, and a kernel profile of the C++ trainer.
# usage (via gpurun): bash tools/gpu_cpp.sh TAG
TAG=${1:-cpp}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=gpurun_out/cpp_$TAG.log; : > $L
timeout -k 10 300 python -u -m pytest tests/test_native_pipeline.py tests/test_cpp_host_blocks.py tests/test_cpp_host_api.py -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for B in 256 64; do
  timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch $B --steps 30 --bench >> $L 2>&1 || exit $?
  timeout -k 10 240 python bench.py --batch $B --graph 0 --steps 30 --warmup 5 >> $L 2>&1 || exit $?
done
timeout -k 10 300 dcnn_amd/bin/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 >> $L 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cpp$TAG -o run -- $R/dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch 256 --steps 10 --bench > $R/gpurun_out/prof_cpp$TAG.log 2>&1 || exit $?
cd $R && DB=$(find gpurun_out/prof_cpp$TAG -name 'run_results.db' -print -quit) && python tools/prof_summary.py $DB > gpurun_out/prof_cpp$TAG.md 2>&1
exit 0
