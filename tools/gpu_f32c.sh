#!/bin/bash
# fp32 split-precision halo convs: targeted tests, benches (concat on / off), kernel profile.
TAG=${1:-f32c}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -q -x -rf \
  -k "fp32 or split3 or dense_fp32" --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/t_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_$TAG.log
case $rc in 0|1) ;; *) exit $rc ;; esac
O=gpurun_out/bench_$TAG.jsonl; : > $O
for c in 1 0; do
  DCNN_F32_CONCAT=$c timeout -k 10 240 python bench.py --model resnet9_cifar10 --dtype fp32 --batch 128 --steps 20 --warmup 5 2>>gpurun_out/bench_$TAG.err | grep '^{' | sed "s/^{/{\"concat\": $c, /" >> $O || exit $?
  DCNN_F32_CONCAT=$c timeout -k 10 240 python bench.py --dtype fp32 --batch 256 --steps 20 --warmup 5 2>>gpurun_out/bench_$TAG.err | grep '^{' | sed "s/^{/{\"concat\": $c, /" >> $O || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model resnet9_cifar10 --dtype fp32 --batch 128 --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
