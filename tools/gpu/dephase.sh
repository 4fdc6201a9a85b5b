#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in 0 40 80 160 0; do echo "== dephase $d"; DCNN_H3_DEPHASE=$d timeout -k 10 120 python benchmarks/conv_bench.py --shapes l1.c,l2.c --iters 20 2>&1 | grep -E "fwd|dgrad" || exit 1; done
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in 1 2; do for d in 0 80; do
  x=$(DCNN_H3_DEPHASE=$d timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  echo "dephase $d r18 $x"; done; done
