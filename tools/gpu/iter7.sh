#!/bin/bash
# RCCL link pair selftest + native pipeline GPU tests + IPC hand-off modes (ResNet-50 4-stage 1F1B)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=gpurun_out/it7.log; : > $L
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider tests/test_cpp_host_api.py::test_selftest_gpu_matches_cpu_backend tests/test_native_pipeline.py -m gpu >> $L 2>&1 || { tail -40 $L; exit 1; }
for E in host event flag host event; do
  echo "== DCNN_IPC_HANDOFF=$E" >> $L
  DCNN_IPC_HANDOFF=$E timeout -k 10 300 dcnn_amd/bin/pipeline_coordinator --spawn 4 --model resnet50_tiny_imagenet --input 3,64,64 --classes 200 --device GPU:0 --batch 256 --microbatches 8 --schedule 1f1b --steps 8 --bench 2 --transport ipc >> $L 2>&1 || { tail -40 $L; exit 1; }
done
grep -E "PASSED|FAILED|==|img/s|images/sec" $L | cut -c1-200
