#!/bin/bash
# Generic A/B of kernel switches: for each "VAR=value ..." setting (or "-" for the defaults) run the
# per-shape conv_bench with the given arguments and the headline bench, all on one box.
# usage (via gpurun): bash tools/gpu_ab.sh TAG "--set r50 --shapes r1.c3 --only fwd" "DCNN_X=0" "-"
# (replaces the round-3 one-off scripts: g1s store paths / occupancy, hconv3 8x8, hwgrad tap split)
# AB_BENCH="--model resnet50_tiny_imagenet --batch 32": extra bench.py arguments
TAG=${1:-ab}; CB=${2:-}; shift 2
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for E in "$@"; do
  [ "$E" = "-" ] && E=""
  echo "== ${E:-defaults}" >> gpurun_out/ab_$TAG.log
  if [ -n "$CB" ]; then
    env $E timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --iters 20 $CB >> gpurun_out/ab_$TAG.log 2>&1 || exit $?
  fi
  env $E timeout -k 10 240 python bench.py --steps 30 --warmup 5 ${AB_BENCH:-} >> gpurun_out/ab_$TAG.log 2>&1 || exit $?
done
