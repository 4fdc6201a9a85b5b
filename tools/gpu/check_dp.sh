set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/pg_capture_probe.py --rounds 30 --drain > gpurun_out/probe_drain.log 2>&1 && echo "drain ok" &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_cpp_dp.py tests/test_device_loader.py tests/test_cpp_host_blocks.py tests/test_cpp_host_api.py tests/test_gpu_dp.py tests/test_gpu_rccl.py -m gpu > gpurun_out/t1.log 2>&1 && echo "tests ok" &&
timeout -k 10 300 python bench.py --steps 30 --warmup 8 > gpurun_out/bench1.log 2>&1 && cat gpurun_out/bench1.log | tail -1 &&
timeout -k 10 120 python -u tools/pg_capture_probe.py --rounds 30 > gpurun_out/probe_nodrain.log 2>&1; echo "nodrain rc=$?"
