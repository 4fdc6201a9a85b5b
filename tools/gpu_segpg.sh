#!/bin/bash
# world-1 process group with forced collectives: segmented vs whole-step capture (bench --pg)
TAG=${1:-segpg}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/segpg_$TAG.log; : > $L
for r in 1 2; do for C in 0 1; do
  echo "== DCNN_DP_CAPTURE=$C" >> $L
  DCNN_DP_FORCE_COLLECTIVES=1 DCNN_DP_CAPTURE=$C timeout -k 10 200 python bench.py --pg --steps 40 --warmup 8 >> $L 2>&1 || exit $?
done; done
