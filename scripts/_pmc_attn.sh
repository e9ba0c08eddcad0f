#!/bin/bash
# PMC passes over the K8 attention kernels at the GPT-2 medium shape (B128 would be slow: B32)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export ATTN_SHAPE=32,1024,16,16,64 ATTN_ITERS=3
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU -d $R/gpurun_out/pmc_attn5a -o run -- python3 $R/bench/attn_prof.py > $R/gpurun_out/pmc_attn5a.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_WAVES -d $R/gpurun_out/pmc_attn5b -o run -- python3 $R/bench/attn_prof.py > $R/gpurun_out/pmc_attn5b.log 2>&1
