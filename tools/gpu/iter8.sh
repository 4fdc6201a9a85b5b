#!/bin/bash
# IPC transport: message vs ipc (device wait) vs ipc (host wait), per-step losses
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/it8.log; : > $L
run() { timeout -k 10 120 dcnn_amd/bin/pipeline_coordinator --spawn 3 --model resnet9_cifar10 --device GPU:0 --input 3,32,32 --classes 10 --batch 64 --microbatches 4 --steps 6 --schedule 1f1b --json "$@"; }
echo "== message" >> $L; run --transport message >> $L 2>&1 || exit 1
echo "== ipc device wait" >> $L; run --transport ipc >> $L 2>&1 || exit 1
echo "== ipc host wait" >> $L; DCNN_IPC_DEVICE_WAIT=0 run --transport ipc >> $L 2>&1 || exit 1
echo "== ipc device wait, eager stages" >> $L; DCNN_STAGE_GRAPHS=0 run --transport ipc >> $L 2>&1 || exit 1
echo "== message, eager stages" >> $L; DCNN_STAGE_GRAPHS=0 run --transport message >> $L 2>&1 || exit 1
grep -E "^==|loss" $L | cut -c1-120 || true
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet18 --batch 256 > gpurun_out/bn_bw_r18.md 2>&1 || { tail -20 gpurun_out/bn_bw_r18.md; exit 1; }
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet50 --batch 256 > gpurun_out/bn_bw_r50.md 2>&1 || { tail -20 gpurun_out/bn_bw_r50.md; exit 1; }
cat gpurun_out/bn_bw_r18.md gpurun_out/bn_bw_r50.md
