#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -rf > gpurun_out/t5.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t5.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 > gpurun_out/conv5.log 2>&1 || exit $?
for B in 256 512; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 1 --batch $B >> gpurun_out/b5.log 2>&1 || exit $?; done
