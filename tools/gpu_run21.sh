#!/bin/bash
# opaque LDS DMA in hwgrad + t2 (no compiler vmcnt(0) before the tr reads): suite, wgrad bench, bench
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/t21.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only wgrad > gpurun_out/c21.log 2>&1 || exit $?
DCNN_HWGRAD=0 timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only wgrad > gpurun_out/c21b.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b21.log 2>&1 || exit $?
