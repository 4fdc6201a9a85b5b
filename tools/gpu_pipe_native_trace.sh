#!/bin/bash
# Kernel trace of the all-native pipeline on one GPU: 4 network_worker processes, each started
# directly under its own rocprofv3 (no profiled process starts another program), driven by the
# native coordinator (ResNet-50, batch 256, 8 micro-batches, 1F1B, IPC transport); GPU busy /
# idle per step from the merged traces (tools/gpu_busy.py).
# usage (via gpurun): bash tools/gpu_pipe_native_trace.sh TAG
TAG=${1:-pnt}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=$R/gpurun_out/pnt_$TAG.log; : > $L
PIDS=()
for i in 0 1 2 3; do
  P=$((29400 + i))
  (cd /tmp && exec timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/pnt_$TAG/w$i -o run -- $R/dcnn_amd/bin/network_worker $P > $R/gpurun_out/pnt_${TAG}_w$i.log 2>&1) &
  PIDS+=($!)
done
sleep 20
timeout -k 10 240 dcnn_amd/bin/pipeline_coordinator --workers 127.0.0.1:29400,127.0.0.1:29401,127.0.0.1:29402,127.0.0.1:29403 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 --transport ipc --partitioner flops >> $L 2>&1; rc=$?
for p in "${PIDS[@]}"; do wait $p; done
[ $rc -eq 0 ] || exit $rc
DBS=$(find gpurun_out/pnt_$TAG -name 'run_results.db' | sort)
python tools/gpu_busy.py $DBS --steps 4 --opt-per-step 4 >> $L 2>&1
