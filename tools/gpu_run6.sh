#!/bin/bash
# bench at several per-GPU batches + rocprof kernel stats of the flagship step
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for B in 256 512 1024; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch $B >> gpurun_out/b6.log 2>&1 || exit $?; done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof6 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --batch 256 > $GRAFT_REPO_ROOT/gpurun_out/prof6.log 2>&1
