#!/bin/bash
# hwgrad fixed cost: 16+1 = no tiles (prologue + epilogue without stores), 16 = no tiles with stores
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in 17 16 19; do
cd /tmp && DCNN_HWGRAD_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof23_$d -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c > $GRAFT_REPO_ROOT/gpurun_out/prof23_$d.log 2>&1 || exit $?
done
