#!/bin/bash
# conv kernel spot check: halo / gathered-GEMM / strided tests, then the headline bench (both engines)
TAG=${1:-quick}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/quick_$TAG.log; : > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_hconv3.py tests/test_gpu_geometry.py tests/test_gpu_model.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $L 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 40 --warmup 8 --engine python >> $L 2>&1 || exit $?
