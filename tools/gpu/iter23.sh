#!/bin/bash
# BatchNorm apply passes: channel-block index by mask when C / 8 is a power of two — tests, R18 table, A/B vs HEAD
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=gpurun_out/it23.log; : > $L
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet18 --batch 256 > gpurun_out/bn_bw_r18.md 2>&1 || exit 1
grep -E "^\| l" gpurun_out/bn_bw_r18.md | awk -F'|' '{print $2,$4,$7}' | grep -v copy | tr '\n' ';'; echo
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in 1 2 3; do for v in new old; do LP=; [ $v = old ] && LP=$R/tools/ab_old
  x=$(LD_LIBRARY_PATH=$LP timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  echo "ab $v r18 $x"; done; done
