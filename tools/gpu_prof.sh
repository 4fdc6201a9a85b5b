#!/bin/bash
# rocprofv3 kernel-trace summary of one bench.py configuration.
# usage (via gpurun): bash tools/gpu_prof.sh TAG [bench.py args...]
TAG=${1:-prof}; shift
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py "$@" > $R/gpurun_out/prof_$TAG.log 2>&1 || exit $?
cd $R && DB=$(find gpurun_out/prof_$TAG -name 'run_results.db' -print -quit) && python tools/prof_summary.py $DB > gpurun_out/prof_$TAG.md 2>&1
