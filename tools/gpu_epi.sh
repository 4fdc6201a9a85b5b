#!/bin/bash
# hconv epilogue change: numerics tests, per-shape conv times, headline bench at 256 / 64
TAG=${1:-epi}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf -x -k "hconv or conv_fwd_dgrad or bnb or epilogue" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --shapes l1.c,l2.c,l3.c,l4.c > gpurun_out/conv_$TAG.txt 2>/dev/null || exit $?
B=gpurun_out/bench_$TAG.jsonl; : > $B
for b in 256 64; do
  timeout -k 10 240 python bench.py --batch $b --steps 30 --warmup 5 2>>gpurun_out/bench_$TAG.err | grep '^{' >> $B || exit $?
done
