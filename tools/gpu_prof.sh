#!/bin/bash
# Bench + kernel-trace profile of one bench.py configuration, with the hot-path purity check.
# usage (via gpurun): bash tools/gpu_prof.sh TAG [bench.py args...]
#   e.g. bash tools/gpu_prof.sh r50b32 --model resnet50_tiny_imagenet --batch 32
TAG=${1:-prof}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py "$@" --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py "$@" --steps 10 --warmup 3 > $R/gpurun_out/prof_$TAG.log 2>&1 || exit $?
cd $R && DB=$(find gpurun_out/prof_$TAG -name 'run_results.db' -print -quit)
python tools/prof_summary.py $DB > gpurun_out/prof_$TAG.md 2>&1
python tools/check_hot_path.py $DB > gpurun_out/hot_$TAG.txt 2>&1
exit 0
