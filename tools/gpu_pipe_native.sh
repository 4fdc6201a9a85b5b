#!/bin/bash
# Native pipeline on one GPU: the native pipeline GPU tests, then 4 native stage processes + the
# native coordinator (ResNet-50, batch 256, 8 micro-batches, 1F1B, IPC transport): per-micro-batch
# hipGraphs on / off, the loss on the last stage's GPU / on the coordinator, FLOP-balanced / naive
# partition.
# usage (via gpurun): bash tools/gpu_pipe_native.sh TAG
TAG=${1:-pn}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/pn_$TAG.log; : > $L
timeout -k 10 500 python -u -m pytest tests/test_native_pipeline.py -m gpu -v -rf --timeout 240 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for V in "1 auto flops" "1 auto naive" "1 0 flops" "0 auto flops"; do
  set -- $V
  echo "== DCNN_STAGE_GRAPHS=$1 --stage-loss $2 --partitioner $3" >> $L
  DCNN_STAGE_GRAPHS=$1 timeout -k 10 300 dcnn_amd/bin/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 --transport ipc --stage-loss $2 --partitioner $3 >> $L 2>&1 || exit $?
done
