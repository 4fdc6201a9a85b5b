#!/bin/bash
# segmented captures in thread_local mode: DP / RCCL / step GPU tests
TAG=${1:-dpfix2}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/dpfix2_$TAG.log; : > $L
timeout -k 10 700 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dp.py tests/test_gpu_arena.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1; rc=$?
echo "pytest rc=$rc" >> $L; exit $rc
