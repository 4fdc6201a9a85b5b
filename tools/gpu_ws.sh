#!/bin/bash
# A/B of the weight-gradient side stream: GPU tests (model + DP + pipeline), bench with it on / off,
# kernel trace of the on variant.
TAG=${1:-ws}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
O=gpurun_out/ws_$TAG.jsonl; : > $O
for v in 1 0 1 0; do
  DCNN_WGRAD_STREAM=$v timeout -k 10 200 python bench.py --steps 40 --warmup 5 2>>gpurun_out/ws_$TAG.err | grep '^{' | sed "s/^{/{\"wgrad_stream\": $v, /" >> $O || exit $?
done
DCNN_WGRAD_STREAM=1 timeout -k 10 200 python bench.py --batch 128 --steps 40 --warmup 5 2>>gpurun_out/ws_$TAG.err | grep '^{' >> $O || exit $?
DCNN_WGRAD_STREAM=1 timeout -k 10 200 python bench.py --batch 64 --steps 40 --warmup 5 2>>gpurun_out/ws_$TAG.err | grep '^{' >> $O || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
