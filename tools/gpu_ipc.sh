#!/bin/bash
# Native pipeline on one GPU: the IPC transport test, then 4 stage processes + the native
# coordinator, inline TCP payloads vs device IPC buffers (ResNet-50, batch 256, 1F1B).
# usage (via gpurun): bash tools/gpu_ipc.sh TAG
TAG=${1:-ipc}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/ipc_$TAG.log; : > $L
timeout -k 10 300 python -u -m pytest tests/test_native_pipeline.py -m gpu -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit $?
for T in message ipc; do
  timeout -k 10 300 dcnn_amd/bin/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 --transport $T >> $L 2>&1 || exit $?
done
