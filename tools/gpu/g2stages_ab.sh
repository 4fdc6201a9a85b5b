#!/bin/bash
# gemm_g2 ring depth: the default rule vs 2 stages everywhere (same box, alternating)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/g2stages.log; : > $L
S=l2.b1c1,l3.b1c1,l4.b1c1,l2.proj,l3.proj,l4.proj
timeout -k 10 120 python benchmarks/conv_bench.py --only fwd --shapes $S --iters 20 >> $L 2>&1 || exit 1
DCNN_G2_STAGES=2 timeout -k 10 120 python benchmarks/conv_bench.py --only fwd --shapes $S --iters 20 >> $L 2>&1 || exit 1
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
B=dcnn_amd/bin/tiny_imagenet_resnet18
for rep in 1 2 3; do for v in def st2; do E=; [ $v = st2 ] && E=2
  x=$(DCNN_G2_STAGES=$E timeout -k 10 300 $B --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  y=$(DCNN_G2_STAGES=$E timeout -k 10 300 $B --device GPU --bench --model resnet50_tiny_imagenet --batch 32 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  echo "ab $v r18 $x r50b32 $y" >> $L; done; done
cat $L
