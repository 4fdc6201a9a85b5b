#!/bin/bash
# hwgrad with the cheap halo loader: numerics + timing (normal / no loads+stores)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k "halo or conv" > gpurun_out/t19.log 2>&1 || exit $?
for d in 0 3; do
cd /tmp && DCNN_HWGRAD_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof19_$d -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c,l2.c,l3.c,l4.c > $GRAFT_REPO_ROOT/gpurun_out/prof19_$d.log 2>&1 || exit $?
done
