#!/bin/bash
# Kernel traces of the ResNet-50 pipeline schedules on one GPU (4 stages): GPU busy / idle per step.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for S in sync 1f1b semi_async; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/pt_$S -o run -- python3 $R/benchmarks/pipeline_bench.py --stages 4 --schedule $S --steps 6 --warmup 3 > $R/gpurun_out/pt_$S.log 2>&1 || exit $?
  cd $R && DB=$(find gpurun_out/pt_$S -name 'run_results.db' -print -quit)
  echo "== $S" >> gpurun_out/pt_busy.txt
  grep '^{' gpurun_out/pt_$S.log >> gpurun_out/pt_busy.txt
  python tools/gpu_busy.py $DB --steps 4 --opt-per-step 4 >> gpurun_out/pt_busy.txt 2>&1
done
