#!/bin/bash
# hwgrad PMC counters (stall breakdown), normal and timing-only (no loads/stores)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for d in 0 3; do
cd /tmp && DCNN_HWGRAD_DBG=$d timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc20_$d -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/conv_bench.py --batch 256 --only wgrad --shapes l1.c --iters 3 > $GRAFT_REPO_ROOT/gpurun_out/pmc20_$d.log 2>&1 || exit $?
done
