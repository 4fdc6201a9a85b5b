#!/bin/bash
# g1s pixel decode on multiply-shift reciprocals: geometry / kernel tests + same-box A/B vs HEAD
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=gpurun_out/it22.log; : > $L
timeout -k 10 1200 python -u -m pytest -x -q --timeout 900 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_g1s.py tests/test_gpu_cpp_geometry.py -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in 1 2 3; do for v in new old; do LP=; [ $v = old ] && LP=$R/tools/ab_old
  x=$(LD_LIBRARY_PATH=$LP timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  y=$(LD_LIBRARY_PATH=$LP timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --model resnet50_tiny_imagenet --batch 32 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  echo "ab $v r18 $x r50b32 $y"; done; done
