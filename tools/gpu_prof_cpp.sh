#!/bin/bash
# rocprofv3 kernel-trace summary of the C++ host API's captured training step (bin/tiny_imagenet_resnet18).
# usage (via gpurun): bash tools/gpu_prof_cpp.sh TAG [trainer args...]
TAG=${1:-cpp}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- $R/dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU "$@" > $R/gpurun_out/prof_$TAG.log 2>&1 || exit $?
cd $R && DB=$(find gpurun_out/prof_$TAG -name 'run_results.db' -print -quit) && python tools/prof_summary.py $DB > gpurun_out/prof_$TAG.md 2>&1
