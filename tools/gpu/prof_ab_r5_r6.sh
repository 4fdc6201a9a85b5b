#!/bin/bash
# same-box rocprofv3 kernel tables of the round-5 (tools/ab_r5) and round-6 C++ headline step
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in r6 r5; do
  B=$R/dcnn_amd/bin; [ $v = r5 ] && B=$R/tools/ab_r5/bin
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/profab_$v -o run -- $B/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 20 --warmup 5 --loss softmax_ce > $R/gpurun_out/profab_$v.log 2>&1) || exit 1
  DB=$(find gpurun_out/profab_$v -name 'run_results.db' -print -quit) && python tools/prof_summary.py $DB > gpurun_out/profab_$v.md 2>&1 || exit 1
  grep "kernel time per step" gpurun_out/profab_$v.md
done
