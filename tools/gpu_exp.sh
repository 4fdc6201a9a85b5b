#!/bin/bash
# Ad-hoc kernel experiments: conv_bench on chosen shapes under env switches, timeline.
# usage (via gpurun): bash tools/gpu_exp.sh TAG
TAG=${1:-exp}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
O=gpurun_out/exp_$TAG.log; : > $O
run() { echo "== $*" >> $O; timeout -k 10 120 env "$@" >> $O 2>&1 || exit $?; }
run DCNN_HCONV3_8=1 DCNN_HCONV_SPLIT=256 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l3.c,l4.c --only fwd
run DCNN_HCONV3_8=1 DCNN_HCONV_SPLIT=512 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l3.c,l4.c --only fwd
run DCNN_HCONV_SPLIT=256 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l3.c,l4.c --only fwd
run DCNN_HCONV_SPLIT=1024 python benchmarks/conv_bench.py --batch 256 --iters 20 --shapes l3.c,l4.c --only fwd
run python benchmarks/hconv3_timeline.py --batch 256 --shapes l1.c,l2.c
run DCNN_HCONV3_8=1 DCNN_HCONV_SPLIT=256 python benchmarks/hconv3_timeline.py --batch 256 --shapes l3.c
exit 0
