#!/bin/bash
# hwgrad ablations: 3 = no global traffic, 7 = +no LDS reads after step 0, 11 = +no MFMA, 15 = neither
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in 0 3 7 11 15; do
cd /tmp && DCNN_HWGRAD_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof22_$d -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c > $GRAFT_REPO_ROOT/gpurun_out/prof22_$d.log 2>&1 || exit $?
done
cd /tmp && DCNN_HWGRAD_BLOCKS=128 DCNN_HWGRAD_DBG=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof22_b128 -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c > $GRAFT_REPO_ROOT/gpurun_out/prof22_b128.log 2>&1
