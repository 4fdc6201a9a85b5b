#!/bin/bash
# hwgrad2 tap-split (8 waves, DCNN_HWGRAD_TS=2) vs the 4-wave kernel: tests, per-shape wgrad, bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for T in 2 3; do
  DCNN_HWGRAD_TS=$T timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "halo_wgrad or conv_fwd_dgrad_wgrad or deferred" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_hwts$T.log 2>&1 || exit $?
done
for T in 2 3; do
  echo "== TS=$T" >> gpurun_out/cb_hwts.log
  DCNN_HWGRAD_TS=$T timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l1.c,l2.c,l3.c,l4.c --only wgrad >> gpurun_out/cb_hwts.log 2>&1 || exit $?
done
for T in 2 3 2 3; do
  echo "== TS=$T" >> gpurun_out/b_hwts.log
  DCNN_HWGRAD_TS=$T timeout -k 10 240 python bench.py --steps 30 --warmup 5 >> gpurun_out/b_hwts.log 2>&1 || exit $?
done
