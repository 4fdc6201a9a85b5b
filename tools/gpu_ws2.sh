#!/bin/bash
# stride-2 halo weight gradient: numerics, per-shape times vs gemm_t2, headline step (Python engine)
TAG=${1:-ws2}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=gpurun_out/ws2_$TAG.log; : > $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "stride2 or strided" >> $L 2>&1 || exit $?
for P in 0 1; do
  echo "== hwgrad_s2 $P" >> $L
  timeout -k 10 120 python benchmarks/conv_bench.py --batch 256 --iters 20 --only wgrad --shapes l2.b1c1,l3.b1c1,l4.b1c1 --hwgrad-s2 $P >> $L 2>&1 || exit $?
  timeout -k 10 120 python benchmarks/conv_bench.py --batch 64 --iters 20 --only wgrad --shapes l2.b1c1,l3.b1c1,l4.b1c1 --hwgrad-s2 $P >> $L 2>&1 || exit $?
  timeout -k 10 120 python benchmarks/conv_bench.py --set r50 --batch 256 --iters 20 --only wgrad --shapes r2.s2 --hwgrad-s2 $P >> $L 2>&1 || exit $?
  timeout -k 10 120 python benchmarks/conv_bench.py --set r50 --batch 32 --iters 20 --only wgrad --shapes r2.s2 --hwgrad-s2 $P >> $L 2>&1 || exit $?
done
for r in 1 2; do for P in 0 1; do
  echo "== bench hwgrad_s2 $P" >> $L
  timeout -k 10 200 python -c "import sys, runpy; from dcnn_amd.ops import fusion; fusion.HWGRAD_S2 = bool($P); sys.argv = ['bench.py', '--engine', 'python', '--steps', '40', '--warmup', '8']; runpy.run_path('bench.py', run_name='__main__')" >> $L 2>&1 || exit $?
done; done
