#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -m gpu -rf -x > gpurun_out/t4.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 > gpurun_out/conv4.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 1 --batch 256 > gpurun_out/b4.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4 -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 --graph 0 --batch 256 > gpurun_out/prof4.log 2>&1
