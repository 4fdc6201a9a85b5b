# one perf iteration: GPU correctness of the conv routes (Python + C++ geometry), the headline bench,
# and a kernel-trace table of the C++ step (TAG = $1)
TAG=${1:-iter}
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_geometry.py tests/test_gpu_cpp_geometry.py > gpurun_out/t_$TAG.log 2>&1 || { echo "geometry tests failed"; tail -30 gpurun_out/t_$TAG.log; exit 1; }
echo "geometry ok"
timeout -k 10 300 python bench.py --steps 40 --warmup 8 > gpurun_out/bench_$TAG.log 2>&1 || exit 1
tail -1 gpurun_out/bench_$TAG.log
bash tools/gpu_prof_cpp.sh $TAG --bench --batch 256 --steps 20 --warmup 5 --loss softmax_ce || exit 1
head -30 gpurun_out/prof_$TAG.md
