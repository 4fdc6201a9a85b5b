#!/bin/bash
# weight-stationary hconv: numerics tests first, then per-shape A/B, then the headline bench
TAG=${1:-ws}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -x -k "weight_stationary or conv_fwd_dgrad or wide_tiles or layer4" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || exit $?
O=gpurun_out/convws_$TAG.txt; : > $O
for E in "DCNN_HCONV_WS=0" "DCNN_HCONV_WS=1"; do
  echo "== $E" >> $O
  env $E timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --shapes l1.c >> $O 2>/dev/null || exit $?
  env $E timeout -k 10 200 python benchmarks/conv_bench.py --batch 64 --shapes l1.c >> $O 2>/dev/null || exit $?
done
B=gpurun_out/bench_$TAG.jsonl; : > $B
for b in 256 64; do
  timeout -k 10 240 python bench.py --batch $b --steps 30 --warmup 5 2>>gpurun_out/bench_$TAG.err | grep '^{' >> $B || exit $?
done
