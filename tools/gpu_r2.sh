#!/bin/bash
# Round-2 GPU check: full GPU test suite (no -x: every failure listed), headline bench at
# batch 256/128/64, and a rocprofv3 kernel-stats profile of the batch-256 step.
# usage (via gpurun): bash tools/gpu_r2.sh TAG [skip_tests]
TAG=${1:-r2}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${2:-}" != "skip_tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
fi
O=gpurun_out/bench_$TAG.jsonl; : > $O
for b in 256 128 64; do
  timeout -k 10 240 python bench.py --batch $b --steps 30 --warmup 5 > gpurun_out/cur.out 2>gpurun_out/bench_$TAG.err || exit $?
  grep '^{' gpurun_out/cur.out >> $O
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
