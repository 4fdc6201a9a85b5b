#!/bin/bash
# Full GPU suite, headline bench at 256/128/64, pipeline schedules + PyTorch pipeline baseline,
# kernel profile of the headline step.
TAG=${1:-all}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
O=gpurun_out/bench_$TAG.jsonl; : > $O
for b in 256 128 64; do
  timeout -k 10 240 python bench.py --batch $b --steps 30 --warmup 5 2>>gpurun_out/bench_$TAG.err | grep '^{' >> $O || exit $?
done
P=gpurun_out/pipe_$TAG.jsonl; : > $P
for cfg in "--stages 4 --schedule sync" "--stages 4 --schedule 1f1b" "--stages 8 --schedule semi_async" "--stages 8 --schedule 1f1b"; do
  timeout -k 10 300 python benchmarks/pipeline_bench.py $cfg --steps 10 --warmup 3 2>>gpurun_out/pipe_$TAG.err | grep '^{' >> $P || exit $?
done
for cfg in "--stages 4 --schedule gpipe --mode bf16" "--stages 8 --schedule gpipe --mode bf16" "--stages 4 --schedule 1f1b --mode bf16"; do
  timeout -k 10 400 python -u benchmarks/torch_pipeline_baseline.py $cfg --steps 10 --warmup 3 2>>gpurun_out/pipe_$TAG.err | grep '^{' >> $P || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
