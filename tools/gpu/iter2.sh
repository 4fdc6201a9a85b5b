cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_geometry.py tests/test_gpu_cpp_geometry.py tests/test_gpu_hconv3.py > gpurun_out/t_it2.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_it2.log; exit 1; }
echo "tests ok"
bash tools/gpu/perf_ab.sh defer - DCNN_DEFER_REDUCE=0 || exit 1
bash tools/gpu_prof_cpp.sh it2 --bench --batch 256 --steps 20 --warmup 5 --loss softmax_ce || exit 1
head -40 gpurun_out/prof_it2.md
