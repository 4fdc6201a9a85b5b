#!/bin/bash
# same-box A/B of one environment switch (C++ engine, ResNet-18 b256 and ResNet-50 b32, alternating),
# after the given GPU test files.  usage: bash tools/gpu/ab_env.sh VAR=VALUE REPS [pytest files...]
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
SW=$1; REPS=${2:-3}; shift 2
L=gpurun_out/ab_env.log; : > $L
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider "$@" -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
  tail -1 $L
fi
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in $(seq $REPS); do for v in on off; do
  if [ $v = on ]; then E="env"; else E="env $SW"; fi
  x=$($E timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  y=$($E timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --model resnet50_tiny_imagenet --batch 32 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  echo "ab $v r18 $x r50b32 $y" | tee -a $L; done; done
