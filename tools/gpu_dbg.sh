#!/bin/bash
# backward-BN fusion debug: per-parameter fused/unfused gradient differences under env variants
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for E in "X=0" "DCNN_BNB_POOL=0" "DCNN_HWGRAD_STAGES=2 DCNN_HCONV_BSTAGES=2"; do
  echo "=== $E" >> gpurun_out/dbg.txt
  env $E timeout -k 10 200 python tools/debug_bnb.py >> gpurun_out/dbg.txt 2>&1 || exit $?
done
