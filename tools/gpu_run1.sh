#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -q -m gpu -rf > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --graph 0 --batch 128 > gpurun_out/b1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph 1 --batch 256 >> gpurun_out/b1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --graph 0 --batch 256 --profile >> gpurun_out/b1.log 2>&1
