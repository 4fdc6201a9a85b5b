#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in 1 2 3; do for w in 8 4 16; do
  x=$(DCNN_STAT_WAVES=$w timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  y=$(DCNN_STAT_WAVES=$w timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --model resnet50_tiny_imagenet --batch 32 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  echo "waves $w r18 $x r50b32 $y"; done; done
