#!/bin/bash
# Round-5 GPU pass b: device-loader tests, the C++ per-parameter gradient test, the loader benchmark.
# usage (via gpurun): bash tools/gpu_r5_b.sh TAG
TAG=${1:-b}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ok() { case $1 in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_device_loader.py tests/test_cpp_host_blocks.py::test_cpp_resnet18_gpu_gradients_match_cpu_backend -s > gpurun_out/t_$TAG.log 2>&1; rc=$?
ok $rc || exit $rc
timeout -k 10 600 python -u benchmarks/loader_bench.py --images-per-class 50 --batch 256 --steps 40 > gpurun_out/loader_$TAG.log 2>&1 || exit $?
