#!/bin/bash
# hconv3 co-resident phase-shift sweep: tests, per-shape times per stagger, timeline, bench.
TAG=${1:-sg}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_hconv3.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || exit $?
for S in 0 1 2 3 4 6; do
  echo "== stagger $S" >> gpurun_out/cb_$TAG.log
  timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l1.c,l2.c --v3 1 --stagger $S >> gpurun_out/cb_$TAG.log 2>&1 || exit $?
done
for S in 0 2 4; do
  echo "== stagger $S" >> gpurun_out/tl_$TAG.log
  timeout -k 10 120 python benchmarks/hconv3_timeline.py --batch 256 --shapes l1.c,l2.c --stagger $S >> gpurun_out/tl_$TAG.log 2>&1 || exit $?
done
