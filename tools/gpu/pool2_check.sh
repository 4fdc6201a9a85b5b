#!/bin/bash
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/pool2.log; : > $L
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_cpp_host_blocks.py -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
bash tools/gpu_prof_cpp.sh pool2 --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in 1 2; do for mb in 0 48 96 160 256; do
  x=$(DCNN_REDUCE_FLUSH_MB=$mb timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  y=$(DCNN_REDUCE_FLUSH_MB=$mb timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --model resnet50_tiny_imagenet --batch 32 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  echo "flush $mb r18 $x r50b32 $y" | tee -a $L; done; done
bash tools/gpu/ab.sh 2
