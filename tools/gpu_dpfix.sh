#!/bin/bash
# ProcessGroupNCCL event cache off: the DP / RCCL GPU tests (captured steps on both planes), bench
TAG=${1:-dpfix}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/dpfix_$TAG.log; : > $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dp.py tests/test_gpu_pipeline.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider >> $L 2>&1; rc=$?
echo "pytest rc=$rc" >> $L; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --pg --steps 30 --warmup 5 >> $L 2>&1 || exit $?
