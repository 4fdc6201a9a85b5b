#!/bin/bash
# Round-5 GPU pass b: device-loader tests + loader benchmark, gemm_t2 2- vs 3-stage A/B (conv_bench
# weight gradients, then the headline bench both ways), cpp gradient test.
# usage (via gpurun): bash tools/gpu_r5_b.sh TAG
TAG=${1:-b}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ok() { case $1 in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_device_loader.py tests/test_cpp_host_blocks.py::test_cpp_resnet18_gpu_gradients_match_cpu_backend -s > gpurun_out/t_$TAG.log 2>&1; rc=$?
ok $rc || exit $rc
for S in 2 3; do
  timeout -k 10 300 python -u benchmarks/conv_bench.py --batch 256 --iters 20 --only wgrad --t2-stages $S > gpurun_out/conv_${TAG}_t2s$S.log 2>&1 || exit $?
done
for S in 2 3 2 3; do
  timeout -k 10 240 python -c "import sys; sys.argv=['bench.py','--steps','30','--warmup','5']; import dcnn_amd.ops.hip as h; h.kernels().gemm_t2_set_stages($S); import runpy; runpy.run_path('bench.py', run_name='__main__')" >> gpurun_out/bench_${TAG}_t2s$S.log 2>&1 || exit $?
done
timeout -k 10 600 python -u benchmarks/loader_bench.py --images-per-class 50 --batch 256 --steps 40 > gpurun_out/loader_$TAG.log 2>&1 || exit $?
