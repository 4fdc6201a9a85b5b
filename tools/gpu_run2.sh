#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/debug_graph.py > gpurun_out/dbg.log 2>&1; echo "rc=$?" >> gpurun_out/dbg.log
timeout -k 10 600 python -m pytest tests/test_gpu_model.py -q -m gpu -rf > gpurun_out/t2.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o prof --output-format csv -- python bench.py --steps 10 --warmup 3 --graph 0 --batch 256 > gpurun_out/prof1.log 2>&1
echo "prof rc=$?" >> gpurun_out/prof1.log
