#!/bin/bash
# headline bench x3 + BN tables after the C-dependent prologue width
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet18 --batch 256 > gpurun_out/bn_bw_r18.md 2>&1 || { tail -20 gpurun_out/bn_bw_r18.md; exit 1; }
timeout -k 10 300 python -u benchmarks/bn_bench.py --vec-only --model resnet50 --batch 256 > gpurun_out/bn_bw_r50.md 2>&1 || { tail -20 gpurun_out/bn_bw_r50.md; exit 1; }
for r in 1 2 3; do timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'])" || exit 1; done
grep -E "^\| l" gpurun_out/bn_bw_r18.md | awk -F'|' '{print $2,$4,$7}'
grep -E "l3.w|l4.w" gpurun_out/bn_bw_r50.md | awk -F'|' '{print $2,$4,$7}'
