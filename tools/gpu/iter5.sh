cd $GRAFT_REPO_ROOT
DCNN_G2_SPLITK=2 timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_cpp_geometry.py -k "matches_fp32" > gpurun_out/t_it5.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_it5.log; exit 1; }
echo "tests ok"
AB_MODEL=resnet50_tiny_imagenet AB_BATCH=32 bash tools/gpu/perf_ab.sh tile32 - DCNN_G2_SPLITK=0 DCNN_G2_SPLITK=2 || exit 1
