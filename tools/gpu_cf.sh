#!/bin/bash
# hconv3 checks + C++ path + fp32 path in one call; stops at the first GPU fault / abort / time limit
cd "$GRAFT_REPO_ROOT"
ok() { case $1 in 0|1) return 0;; *) return 1;; esac; }
bash tools/gpu_h3.sh "h$1"; rc=$?; ok $rc || exit $rc
bash tools/gpu_cpp.sh "$1"; rc=$?; ok $rc || exit $rc
bash tools/gpu_f32.sh "$2"
