cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_cpp_geometry.py tests/test_cpp_host_blocks.py tests/test_cpp_host_api.py -m gpu > gpurun_out/t_it3.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_it3.log; exit 1; }
echo "tests ok"
bash tools/gpu/perf_ab.sh fold - DCNN_STAT_FOLD=1 || exit 1
AB_MODEL=resnet50_tiny_imagenet AB_BATCH=32 bash tools/gpu/perf_ab.sh fold50 - DCNN_STAT_FOLD=1 || exit 1
bash tools/gpu_prof_cpp.sh it3 --bench --batch 256 --steps 20 --warmup 5 --loss softmax_ce || exit 1
head -30 gpurun_out/prof_it3.md
