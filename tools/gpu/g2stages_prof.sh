#!/bin/bash
# per-kernel traces of the C++ ResNet-18 b256 step: default gemm_g2 ring rule vs 2 stages
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_prof_cpp.sh def --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
DCNN_G2_STAGES=2 bash tools/gpu_prof_cpp.sh st2 --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
DCNN_G2_STAGES=3 bash tools/gpu_prof_cpp.sh st3 --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
