#!/bin/bash
# Round-5 GPU pass: the new GPU tests, the production-geometry test, per-shape conv timings (all
# ResNet-18 shapes), the headline bench's per-layer profile, four PMC passes that split the conv
# kernels' wave cycles by cause (tools/pmc_table.py), and the RCCL capture probe.
# A failing test (pytest rc 1) does not stop the run; a crash, abort or timeout does.
# usage (via gpurun): bash tools/gpu_r5_a.sh TAG
TAG=${1:-a}
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ok() { case $1 in 0|1) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dp.py::test_gpu_dp_bf16_wire_captured_world1 \
  tests/test_cpp_host_blocks.py::test_cpp_resnet18_gpu_gradients_match_cpu_backend -s > gpurun_out/t_$TAG.log 2>&1; rc=$?
ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 800 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_geometry.py -s > gpurun_out/tg_$TAG.log 2>&1; rc=$?
ok $rc || exit $rc
timeout -k 10 300 python -u benchmarks/conv_bench.py --batch 256 --iters 20 > gpurun_out/conv_$TAG.log 2>&1 || exit $?
timeout -k 10 240 python bench.py --steps 10 --warmup 3 --profile > gpurun_out/layers_$TAG.log 2>&1 || exit $?
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"
P3="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU"
P4="SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
n=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  n=$((n+1))
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc5_${TAG}_$n -o run -- python3 $R/benchmarks/conv_bench.py --batch 256 --iters 3 > $R/gpurun_out/pmc5_${TAG}_$n.log 2>&1) || exit $?
done
F=""
for n in 1 2 3 4; do F="$F $(find gpurun_out/pmc5_${TAG}_$n -name '*counter_collection.csv' -print -quit)"; done
python tools/pmc_table.py --match hconv3,hwgrad2,gemm_g2,gemm_t2,g1s $F > gpurun_out/pmc5_$TAG.md 2>&1
timeout -k 10 900 python -u tools/rccl_capture_probe.py > gpurun_out/probe_$TAG.log 2>&1
