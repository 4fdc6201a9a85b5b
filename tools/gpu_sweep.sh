#!/bin/bash
# GPU test suite + smoke, then one 1-GPU bench per env setting (A/B/C... sweeps of the DCNN_*
# kernel switches). usage (via gpurun): bash tools/gpu_sweep.sh TAG "ENV_1" "ENV_2" ...
# each ENV_i is a space-separated list of VAR=value (use X=0 for "defaults")
TAG=${1:-sweep}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
i=0
for E in "$@"; do
  env $E timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/b_${TAG}_$i.log 2>&1 || exit $?
  echo "$E :: $(tail -1 gpurun_out/b_${TAG}_$i.log)" >> gpurun_out/sweep_$TAG.txt
  i=$((i+1))
done
cat gpurun_out/sweep_$TAG.txt
