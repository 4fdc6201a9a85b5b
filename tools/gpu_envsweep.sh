#!/bin/bash
# Headline bench per env setting and batch: bash tools/gpu_envsweep.sh TAG "BATCHES" "ENV_1" "ENV_2" ...
# (each ENV_i a space-separated VAR=value list, X=0 for defaults); lines in gpurun_out/sweep_TAG.txt
TAG=${1:-sw}; BS=${2:-256}; shift 2
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
O=gpurun_out/sweep_$TAG.txt; : > $O
for E in "$@"; do
  for b in $BS; do
    env $E timeout -k 10 240 python bench.py --steps 30 --warmup 5 --batch $b > gpurun_out/cur.out 2>&1 || exit $?
    echo "$E b=$b :: $(grep '^{' gpurun_out/cur.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> $O
  done
done
cat $O
