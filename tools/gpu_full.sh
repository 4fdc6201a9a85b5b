#!/bin/bash
# full GPU test suite + smoke + 1-GPU benches (via gpurun): bash tools/gpu_full.sh TAG [nobench]
TAG=${1:-full}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
# a fault / abort / time limit ends the call here
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
if [ "$2" != "nobench" ]; then
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/b_$TAG.log 2>&1 || exit $?
  timeout -k 10 240 python bench.py --batch 64 --steps 30 --warmup 5 > gpurun_out/b64_$TAG.log 2>&1 || exit $?
fi
exit $rc
