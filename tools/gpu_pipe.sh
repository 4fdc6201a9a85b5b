#!/bin/bash
# Pipeline runtime check: pipeline GPU tests, then ResNet-50 pipeline throughput (graph + eager)
# against the single-GPU hipGraph step at the micro-batch size.
# usage (via gpurun): bash tools/gpu_pipe.sh TAG [skip_tests]
TAG=${1:-pipe}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${2:-}" != "skip_tests" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -v -rf --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
fi
O=gpurun_out/pipe_$TAG.jsonl; : > $O
timeout -k 10 200 python bench.py --model resnet50_tiny_imagenet --batch 32 --steps 40 --warmup 5 2>>gpurun_out/pipe_$TAG.err | grep '^{' >> $O || exit $?
for cfg in "--stages 1 --schedule sync" "--stages 4 --schedule sync" "--stages 4 --schedule semi_async" "--stages 8 --schedule semi_async" "--stages 4 --schedule sync --no-graph"; do
  timeout -k 10 300 python benchmarks/pipeline_bench.py $cfg --steps 10 --warmup 3 2>>gpurun_out/pipe_$TAG.err | grep '^{' >> $O || exit $?
done
