#!/bin/bash
# PMC pass over a conv_bench subset. usage: bash tools/gpu_pmc.sh TAG "SHAPES" "OPS" "COUNTERS" [conv_bench args]
# (e.g. "--set r50" for the ResNet-50 shapes)
TAG=$1; SHAPES=$2; OPS=$3; CNT=$4; EXTRA=${5:-}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -s KILL 30 rocprofv3 -L > $R/gpurun_out/pmc_list.txt 2>&1
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d $R/gpurun_out/pmc_$TAG -o run -- python3 $R/benchmarks/conv_bench.py --batch 256 --iters 3 --eager --shapes $SHAPES --only $OPS $EXTRA > $R/gpurun_out/pmc_$TAG.log 2>&1
