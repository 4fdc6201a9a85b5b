#!/bin/bash
# hconv3 gutter-layout (4x4 maps) 2-bit swizzle: tests + same-box kernel tables new vs HEAD (tools/ab_old)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
L=gpurun_out/it21.log; : > $L
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_hconv3.py tests/test_gpu_kernels.py tests/test_gpu_cpp_geometry.py tests/test_gpu_model.py -m gpu >> $L 2>&1 || { tail -30 $L; exit 1; }
tail -1 $L
for v in new old; do
  LP=; [ $v = old ] && LP=$R/tools/ab_old
  (cd /tmp && LD_LIBRARY_PATH=$LP timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/swz_$v -o run -- $R/dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 20 --warmup 5 --loss softmax_ce > $R/gpurun_out/swz_$v.log 2>&1) || exit 1
  DB=$(find gpurun_out/swz_$v -name 'run_results.db' -print -quit) && python tools/prof_summary.py $DB > gpurun_out/swz_$v.md 2>&1 || exit 1
  echo "== $v"; grep -E "hconv3_kernel<4, 1, 16, 7|kernel time per step" gpurun_out/swz_$v.md
done
val() { python -c "import json,sys; d=[json.loads(l) for l in sys.stdin.read().splitlines() if l.startswith('{')][-1]; print(d['value'], d.get('loss'))"; }
for rep in 1 2; do for v in new old; do LP=; [ $v = old ] && LP=$R/tools/ab_old
  x=$(LD_LIBRARY_PATH=$LP timeout -k 10 300 dcnn_amd/bin/tiny_imagenet_resnet18 --device GPU --bench --batch 256 --steps 40 --warmup 8 --loss softmax_ce | val) || exit 1
  echo "ab $v $x"; done; done
