#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_cpp_host_blocks.py -k "stem_bn_fold or teacher or gradients_match" -m gpu > gpurun_out/stemfold_t.log 2>&1 || { tail -30 gpurun_out/stemfold_t.log; exit 1; }
tail -1 gpurun_out/stemfold_t.log
bash tools/gpu_prof_cpp.sh fold --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
DCNN_STEM_BNT_BLOCKS=1024 bash tools/gpu_prof_cpp.sh fold1024 --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
DCNN_STEM_BN_FOLD=0 bash tools/gpu_prof_cpp.sh nofold --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
