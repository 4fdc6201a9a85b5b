#!/bin/bash
# C++ host API fusion parity: the C++ GPU tests (per-parameter gradients, captured-step replay,
# trainer), the C++ trainer vs bench.py at batch 256 and a kernel profile of the C++ step.
# usage (via gpurun): bash tools/gpu_cpp_fuse.sh TAG
TAG=${1:-fuse}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=gpurun_out/cppf_$TAG.log; : > $L
timeout -k 10 400 python -u -m pytest tests/test_cpp_host_blocks.py tests/test_cpp_host_api.py -m gpu -v -rf --timeout 240 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch 256 --steps 40 --bench >> $L 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 40 --warmup 5 >> $L 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cpp$TAG -o run -- $R/dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --batch 256 --steps 30 --bench > $R/gpurun_out/prof_cpp$TAG.log 2>&1 || exit $?
cd $R && DB=$(find gpurun_out/prof_cpp$TAG -name 'run_results.db' -print -quit) && python tools/prof_summary.py $DB > gpurun_out/prof_cpp$TAG.md 2>&1
exit 0
