#!/bin/bash
# hwgrad timing experiments: no stores / no loads / neither
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in 0 1 2 3; do
cd /tmp && DCNN_HWGRAD_DBG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof18_$d -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c,l4.c > $GRAFT_REPO_ROOT/gpurun_out/prof18_$d.log 2>&1 || exit $?
done
