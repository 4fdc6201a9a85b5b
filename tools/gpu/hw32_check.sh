#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/hw32.log; : > $L
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_geometry.py tests/test_gpu_cpp_geometry.py tests/test_cpp_host_blocks.py -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
bash tools/gpu_prof_cpp.sh hw32 --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
cp dcnn_amd/libdcnn.so /tmp/new.so
bash tools/gpu/ab.sh 2
