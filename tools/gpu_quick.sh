#!/bin/bash
# Quick GPU iteration: selected GPU tests (pytest -k expression), batch-256 bench, kernel profile.
# usage (via gpurun): bash tools/gpu_quick.sh TAG "<pytest -k expr>" [files...]
TAG=${1:-q}; K=${2:-}; shift 2; FILES=${@:-tests}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest $FILES -m gpu -q -rf -k "$K" --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
  case $rc in 0|1|5) ;; *) exit $rc ;; esac
fi
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
