#!/bin/bash
# halo wgrad with software-pipelined fragment reads: numerics + per-kernel split
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "halo or conv" > gpurun_out/t17.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 --only wgrad > gpurun_out/c17.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof17 -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c,l2.c,l3.c,l4.c > $GRAFT_REPO_ROOT/gpurun_out/prof17.log 2>&1
