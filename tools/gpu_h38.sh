#!/bin/bash
# hconv3 on 8x8 maps (DCNN_HCONV3_8=1): tests, per-shape l3 times on / off, whole-step benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
DCNN_HCONV3_8=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_hconv3.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_h38.log 2>&1 || exit $?
for E in 0 1; do
  echo "== DCNN_HCONV3_8=$E" >> gpurun_out/cb_h38.log
  DCNN_HCONV3_8=$E timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l3.c >> gpurun_out/cb_h38.log 2>&1 || exit $?
  DCNN_HCONV3_8=$E timeout -k 10 200 python benchmarks/conv_bench.py --batch 64 --iters 20 --shapes l3.c >> gpurun_out/cb_h38.log 2>&1 || exit $?
  DCNN_HCONV3_8=$E timeout -k 10 240 python bench.py --steps 30 --warmup 5 >> gpurun_out/b_h38.log 2>&1 || exit $?
done
