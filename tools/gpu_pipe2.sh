#!/bin/bash
# Pipeline schedules incl. 1F1B + the same-box PyTorch pipeline baseline.
TAG=${1:-pipe2}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -v -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
O=gpurun_out/pipe_$TAG.jsonl; : > $O
for cfg in "--stages 4 --schedule sync" "--stages 4 --schedule 1f1b" "--stages 8 --schedule semi_async" "--stages 8 --schedule 1f1b"; do
  timeout -k 10 300 python benchmarks/pipeline_bench.py $cfg --steps 10 --warmup 3 2>>gpurun_out/pipe_$TAG.err | grep '^{' >> $O || exit $?
done
for cfg in "--stages 4 --schedule gpipe --mode bf16" "--stages 8 --schedule gpipe --mode bf16" "--stages 4 --schedule 1f1b --mode bf16" "--stages 4 --schedule gpipe --mode fp32"; do
  timeout -k 10 400 python benchmarks/torch_pipeline_baseline.py $cfg --steps 10 --warmup 3 2>>gpurun_out/pipe_$TAG.err | grep '^{' >> $O || exit $?
done
