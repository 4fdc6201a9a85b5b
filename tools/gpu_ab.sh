#!/bin/bash
# GPU test suite + smoke, then bench A/B over one env switch, then a kernel profile of B.
# usage (via gpurun): bash tools/gpu_ab.sh TAG "ENV_A" "ENV_B"
TAG=${1:-ab}; A=${2:-X=0}; B=${3:-X=1}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
env $A timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_${TAG}_a.log 2>&1 || exit $?
env $B timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_${TAG}_b.log 2>&1 || exit $?
cd /tmp && env $B timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
