#!/bin/bash
# round-6 end check: full GPU suite, smoke, headline bench, kernel tables (R18 b256, R50 b32)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/t_final.log 2>&1
rc=$?; tail -3 gpurun_out/t_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_final.log 2>&1 || exit 1
tail -1 gpurun_out/bench_final.log
bash tools/gpu_prof_cpp.sh r18_r6_final --bench --batch 256 --steps 20 --warmup 8 --loss softmax_ce || exit 1
bash tools/gpu_prof_cpp.sh r50_r6_final --bench --model resnet50_tiny_imagenet --batch 32 --steps 20 --warmup 8 --loss softmax_ce || exit 1
