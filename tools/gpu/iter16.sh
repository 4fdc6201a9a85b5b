#!/bin/bash
# multi_splitk_reduce entry search: kernel table + bench
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_prof_cpp.sh r18_red --model resnet18_tiny_imagenet --batch 256 --steps 20 --warmup 5 --loss softmax_ce --bench || exit 1
grep -E "multi_splitk|kernel time per step" gpurun_out/prof_r18_red.md
for r in 1 2; do timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'])" || exit 1; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -m gpu -k "splitk or reduce or wgrad" 2>&1 | tail -2
