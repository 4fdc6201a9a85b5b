#!/bin/bash
# Data-parallel step checks on one GPU: DP GPU tests, then bench without a process group, with an
# RCCL world-1 group and the collectives captured in the step graph, and with the segmented capture.
# usage (via gpurun): bash tools/gpu_dp.sh TAG
TAG=${1:-dp}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -m gpu -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
O=gpurun_out/dp_$TAG.jsonl; : > $O
timeout -k 10 200 python bench.py --steps 30 --warmup 5 2>>gpurun_out/dp_$TAG.err | grep '^{' >> $O || exit $?
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --pg 2>>gpurun_out/dp_$TAG.err | grep '^{' >> $O || exit $?
DCNN_DP_CAPTURE=0 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --pg 2>>gpurun_out/dp_$TAG.err | grep '^{' >> $O || exit $?
