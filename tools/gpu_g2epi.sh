#!/bin/bash
# gemm_g2 epilogue change: g2 / strided / model numerics, then R18 b256 kernel table + bench
TAG=${1:-g2epi}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/g2epi_$TAG.log; : > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_conv_routing.py -m gpu -q -x --timeout 200 --timeout-method thread -p no:cacheprovider -k "g2 or strid or dgrad or model or group" >> $L 2>&1 || exit $?
bash tools/gpu_prof.sh r18_$TAG --steps 15 --warmup 5 || exit $?
for r in 1 2; do timeout -k 10 200 python bench.py --steps 40 --warmup 8 --engine python >> $L 2>&1 || exit $?; done
