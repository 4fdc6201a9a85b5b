#!/bin/bash
# BatchNorm WIDE instances: tests, bandwidth tables, same-box A/B (new / HEAD build in tools/ab_old / round 5)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/it19.log; : > $L
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet18 --batch 256 > gpurun_out/bn_bw_r18.md 2>&1 || exit 1
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet50 --batch 256 > gpurun_out/bn_bw_r50.md 2>&1 || exit 1
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in 1 2; do
  for v in new old r5; do
    B=dcnn_amd/bin; LP=
    [ $v = old ] && LP=$GRAFT_REPO_ROOT/tools/ab_old
    [ $v = r5 ] && B=tools/ab_r5/bin
    x=$(LD_LIBRARY_PATH=$LP timeout -k 10 300 $B/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
    y=$(LD_LIBRARY_PATH=$LP timeout -k 10 300 $B/tiny_imagenet_resnet18 --device GPU --bench --model resnet50_tiny_imagenet --batch 32 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
    echo "ab $v r18b256 $x r50b32 $y" | tee -a $L
  done
done
grep -E "^\| l" gpurun_out/bn_bw_r18.md | awk -F'|' '{print $2,$4,$7}'
