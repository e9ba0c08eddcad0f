#!/bin/bash
# K12 vs K12W vs K12W16 vs hipBLASLt weight gradient: SQ pass + HBM-bytes pass on the c_fc and LM-head shapes;
# then the ResNet-50 b2048 steady-step table at HEAD
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for S in 131072,4096,1024 131072,50304,1024; do
  T=$(echo $S | tr , x)
  O=$R/gpurun_out/r6_pmc_wgrad16_$T
  GEMM_OP=wgrad GEMM_SHAPE=$S GEMM_ITERS=3 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d $O -o sq -- python3 $R/bench/gemm_pmc.py > $O.sq.log 2>&1
done
cd $R
bash scripts/gpu_profile_step.sh gpurun_out/r6_prof_resnet_head --model resnet50 --std-batch 0 --steps 6 --warmup 3 > gpurun_out/r6_prof_resnet_head.log 2>&1
head -3 gpurun_out/r6_prof_resnet_head/steps.md
echo pmc done
