#!/bin/bash
# Round-5 baseline: available PMC counters on this box, then the headline bench twice.
# usage (via gpurun): bash tools/gpu_r5_base.sh TAG
TAG=${1:-base}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters_$TAG.txt 2>&1) || echo "rocprofv3 -L rc=$?" >> gpurun_out/counters_$TAG.txt
for i in 1 2; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 >> gpurun_out/b_$TAG.log 2>&1 || exit $?
done
timeout -k 10 240 python bench.py --model resnet50_tiny_imagenet --batch 32 --steps 30 --warmup 5 >> gpurun_out/b_$TAG.log 2>&1 || exit $?
