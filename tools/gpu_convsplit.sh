#!/bin/bash
# conv_bench per-shape times under several env settings: bash tools/gpu_convsplit.sh TAG SHAPES "ENV_1" ...
TAG=${1:-cs}; SH=$2; shift 2
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; O=gpurun_out/convsplit_$TAG.txt; : > $O
for E in "$@"; do
  echo "== $E" >> $O
  env $E timeout -k 10 200 python benchmarks/conv_bench.py --batch 256 --shapes $SH >> $O 2>/dev/null || exit $?
done
cat $O
