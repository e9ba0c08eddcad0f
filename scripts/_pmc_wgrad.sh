#!/bin/bash
# K12 vs K12W vs hipBLASLt weight gradient, one PMC pass per shape (8 SQ + 1 GRBM counters)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for S in 131072,4096,1024 131072,1024,4096; do
  T=$(echo $S | tr , x)
  GEMM_OP=wgrad GEMM_SHAPE=$S timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/r6_pmc_wgrad_$T -o run -- python3 $R/bench/gemm_pmc.py > $R/gpurun_out/r6_pmc_wgrad_$T.log 2>&1
done
echo pmc done
