#!/bin/bash
# K12 vs K12W vs hipBLASLt weight gradient on the GPT-2 c_fc shape: SQ pass, HBM-bytes pass, L2 pass
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
S=131072,4096,1024
T=$(echo $S | tr , x)
O=$R/gpurun_out/r6_pmc_wgrad_s_$T
GEMM_OP=wgrad GEMM_SHAPE=$S timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d $O -o sq -- python3 $R/bench/gemm_pmc.py > $O.sq.log 2>&1
GEMM_OP=wgrad GEMM_SHAPE=$S timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE FETCH_SIZE -d $O -o hbm -- python3 $R/bench/gemm_pmc.py > $O.hbm.log 2>&1
GEMM_OP=wgrad GEMM_SHAPE=$S timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_INSTS_SALU SQ_INSTS_VALU -d $O -o l2 -- python3 $R/bench/gemm_pmc.py > $O.l2.log 2>&1
echo pmc done
