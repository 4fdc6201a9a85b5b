#!/bin/bash
# list gfx950 counters; PMC of hwgrad (clock, MFMA busy, stalls)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp && timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1 || true
cd /tmp && timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc25 -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc25.log 2>&1
