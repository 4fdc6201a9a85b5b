#!/bin/bash
# BatchNorm apply-pass A/B (benchmarks/bn_bench.py), GPU tests touching BatchNorm, headline bench.
TAG=${1:-bn}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/bn_bench.py --batch 256 > gpurun_out/bnb_$TAG.jsonl 2> gpurun_out/bnb_$TAG.err || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
O=gpurun_out/bench_$TAG.jsonl; : > $O
for b in 256 64; do
  timeout -k 10 240 python bench.py --batch $b --steps 30 --warmup 5 2>>gpurun_out/bench_$TAG.err | grep '^{' >> $O || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
