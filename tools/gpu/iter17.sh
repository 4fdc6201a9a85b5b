#!/bin/bash
# hconv3 prologue reorder: GPU tests, per-phase timeline, same-box A/B of the C++ step (old libdcnn
# in tools/ab_old via LD_LIBRARY_PATH: the trainer's RUNPATH yields to it)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/it17.log; : > $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_hconv3.py tests/test_gpu_kernels.py -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
timeout -k 10 300 python -u benchmarks/hconv3_timeline.py --batch 256 --shapes l1.c,l2.c,l4.c >> $L 2>&1 || { tail -30 $L; exit 1; }
for rep in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then LP=$GRAFT_REPO_ROOT/tools/ab_old; else LP=; fi
    x=$(LD_LIBRARY_PATH=$LP timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['loss'])") || exit 1
    echo "ab $v $x" | tee -a $L
  done
done
grep -A12 -i "prologue\|median" $L | head -40
