cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_geometry.py tests/test_gpu_cpp_geometry.py > gpurun_out/t_it4.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/t_it4.log; exit 1; }
echo "tests ok"
AB_MODEL=resnet50_tiny_imagenet AB_BATCH=32 bash tools/gpu/perf_ab.sh splitk50 - DCNN_G2_SPLITK=0 || exit 1
AB_MODEL=resnet50_tiny_imagenet AB_BATCH=256 bash tools/gpu/perf_ab.sh splitk50b - DCNN_G2_SPLITK=0 || exit 1
bash tools/gpu_prof_cpp.sh it4 --model resnet50_tiny_imagenet --bench --batch 32 --steps 20 --warmup 5 --loss softmax_ce || exit 1
head -24 gpurun_out/prof_it4.md
