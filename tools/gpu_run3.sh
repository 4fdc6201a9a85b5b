#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/conv_bench.py --batch 256 > gpurun_out/conv1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d gpurun_out/pmc1 -o pmc --output-format csv -- python benchmarks/conv_bench.py --batch 256 --only fwd --iters 3 > gpurun_out/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM -d gpurun_out/pmc2 -o pmc --output-format csv -- python benchmarks/conv_bench.py --batch 256 --only fwd --iters 3 > gpurun_out/pmc2.log 2>&1
