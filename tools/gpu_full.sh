#!/bin/bash
# Full GPU validation: GPU test suite, smoke(), 1-GPU bench, rocprofv3 kernel stats.
# usage (via gpurun): bash tools/gpu_full.sh TAG
TAG=${1:-full}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
