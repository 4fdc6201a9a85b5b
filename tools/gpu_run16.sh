#!/bin/bash
# kernel-level split of the halo wgrad (hwgrad kernel vs split-K reduce)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof16 -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c,l2.c,l3.c,l4.c > $GRAFT_REPO_ROOT/gpurun_out/prof16.log 2>&1
