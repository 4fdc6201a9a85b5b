#!/bin/bash
# Round-6 PMC passes over the ResNet-18 b256 conv shapes (conv_bench): MFMA busy, wave-cycle shares,
# instruction mix — the gemm_g2 loader after this round's tap-table change, next to the halo kernels
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR"
P3="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU"
n=0
for P in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc6_$n -o run -- python3 $R/benchmarks/conv_bench.py --batch 256 --iters 3 > $R/gpurun_out/pmc6_$n.log 2>&1) || exit 1
done
F=""
for n in 1 2 3; do F="$F $(find gpurun_out/pmc6_$n -name '*counter_collection.csv' -print -quit)"; done
python tools/pmc_table.py --match hconv3,hwgrad2,gemm_g2,gemm_t2,g1s $F > gpurun_out/pmc6.md 2>&1
cat gpurun_out/pmc6.md
