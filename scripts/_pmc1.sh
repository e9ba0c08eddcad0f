set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for S in 8192,8192,8192 131072,4096,1024; do
  T=$(echo $S | tr , x)
  GEMM_SHAPE=$S timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/pmc_$T -o run -- python3 $R/bench/gemm_pmc.py > $R/gpurun_out/pmc_$T.log 2>&1
done
