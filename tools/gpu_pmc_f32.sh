#!/bin/bash
# PMC pass over the exact-fp32 ResNet-9 step (eager, a few steps): MFMA utilisation, issue / wait
# shares per kernel. usage (via gpurun): bash tools/gpu_pmc_f32.sh TAG
TAG=${1:-f32}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CNT="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $R/gpurun_out/pmc_$TAG -o run -- python3 $R/bench.py --model resnet9_cifar10 --dtype fp32 --f32-mode exact --batch 128 --steps 2 --warmup 1 --graph 0 > $R/gpurun_out/pmc_$TAG.log 2>&1 || exit $?
cd $R && F=$(find gpurun_out/pmc_$TAG -name '*counter_collection.csv' -print -quit) && python tools/pmc_summary.py $F > gpurun_out/pmc_$TAG.md 2>&1
