#!/bin/bash
# backward-BN epilogue fusion: kernel-level numerics, then whole-model fused-vs-unfused report
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -q -k bwd_bn_fusion --timeout 120 --timeout-method thread > gpurun_out/t_bnbk.log 2>&1
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python tools/debug_bnb.py > gpurun_out/dbg_bnb.log 2>&1
