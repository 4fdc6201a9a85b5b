#!/bin/bash
# stride-2 halo wgrad, 8-wave variant: numerics, kernel table, headline (both engines)
TAG=${1:-ws2t}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/ws2t_$TAG.log; : > $L
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_geometry.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -k "stride2 or strided or recorded" >> $L 2>&1 || exit $?
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 40 --warmup 8 >> $L 2>&1 || exit $?
  timeout -k 10 200 python bench.py --steps 40 --warmup 8 --engine python >> $L 2>&1 || exit $?
done
bash tools/gpu_prof.sh r18_$TAG --steps 15 --warmup 5
