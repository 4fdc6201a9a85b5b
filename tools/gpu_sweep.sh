#!/bin/bash
# Env-switch sweep of the headline bench: one bench.py run per "VAR=value ..." argument.
# usage (via gpurun): bash tools/gpu_sweep.sh TAG "A=1 B=2" "A=0" ...
TAG=${1:-sw}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for CFG in "$@"; do
  echo "== $CFG" >> gpurun_out/sw_$TAG.log
  env $CFG timeout -k 10 240 python bench.py --steps 30 --warmup 5 >> gpurun_out/sw_$TAG.log 2>&1 || exit $?
done
