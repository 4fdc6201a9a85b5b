#!/bin/bash
# same-box round-5 (tools/ab_r5: binaries + libdcnn of commit 80f2876) vs round-6 (in-tree) runs of
# the headline C++ step (ResNet-18 b256, ResNet-50 b32) and the native 4-stage 1F1B pipeline
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/ab_r5_r6.log; : > $L
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in 1 2; do
  for v in r6 r5; do
    B=dcnn_amd/bin; [ $v = r5 ] && B=tools/ab_r5/bin
    x=$(timeout -k 10 300 $B/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
    echo "r18b256 $v $x" | tee -a $L
    x=$(timeout -k 10 300 $B/tiny_imagenet_resnet18 --device GPU --bench --model resnet50_tiny_imagenet --batch 32 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
    echo "r50b32 $v $x" | tee -a $L
    x=$(timeout -k 10 300 $B/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 --transport ipc | val) || exit 1
    echo "pipe1f1b $v $x" | tee -a $L
  done
done
