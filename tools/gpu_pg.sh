#!/bin/bash
# RCCL world-size-1 checks: the segmented DP graph test and bench with/without a process group.
TAG=${1:-pg}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/b_${TAG}_nopg.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --pg > gpurun_out/b_${TAG}_pg.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --pg --bucket-mb 12 > gpurun_out/b_${TAG}_pg12.log 2>&1
