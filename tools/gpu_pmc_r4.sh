#!/bin/bash
# PMC pass (MFMA busy, issue / wait shares) over the ResNet-18 conv shapes, all three directions.
# usage (via gpurun): bash tools/gpu_pmc_r4.sh TAG
TAG=${1:-pmc4}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CNT="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $R/gpurun_out/pmc_$TAG -o run -- python3 $R/benchmarks/conv_bench.py --batch 256 --iters 3 --eager --shapes l1.c,l2.c,l3.c,l4.c > $R/gpurun_out/pmc_$TAG.log 2>&1 || exit $?
cd $R && F=$(find gpurun_out/pmc_$TAG -name '*counter_collection.csv' -print -quit) && python tools/pmc_summary.py $F > gpurun_out/pmc_$TAG.md 2>&1
