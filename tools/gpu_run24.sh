#!/bin/bash
# hwgrad templated geometry + staged epilogue, unrolled split-K reduce
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t24.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only wgrad > gpurun_out/c24.log 2>&1 || exit $?
for d in 0 17; do
cd /tmp && DCNN_HWGRAD_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof24_$d -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c,l2.c,l3.c,l4.c > $GRAFT_REPO_ROOT/gpurun_out/prof24_$d.log 2>&1 || exit $?
done
