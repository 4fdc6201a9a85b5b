#!/bin/bash
# 1x1 split-K vs hipBLASLt, then the full GPU suite + smoke + headline bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu/iter12.sh > gpurun_out/it12_out.log 2>&1 || { tail -30 gpurun_out/it12.log; exit 1; }
bash tools/gpu/full_suite.sh
