#!/bin/bash
# Full GPU suite (first the files given as arguments, then everything), then the headline bench.
# usage (via gpurun): bash tools/gpu_suite.sh TAG [first test files...]
TAG=${1:-suite}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tf_$TAG.log 2>&1 || exit $?
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ts_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
