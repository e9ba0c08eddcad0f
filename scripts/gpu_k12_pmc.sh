#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT
P2=SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INSTS_SALU,SQ_ACTIVE_INST_ANY,SQ_WAIT_ANY,SQ_WAVES,SQ_INSTS_VMEM
P3=FETCH_SIZE
P4=WRITE_SIZE
cd /tmp && export TMPDIR=/tmp
i=0
for P in $P1 $P2 $P3 $P4; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${P//,/ } --output-format csv -d "$OUT/kpmc$i" -o run -- \
    python3 "$ROOT/bench/k12_pmc.py" > "$OUT/kpmc$i.log" 2>&1 || { tail "$OUT/kpmc$i.log"; exit 3; }
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kpmct" -o run -- \
    python3 "$ROOT/bench/k12_pmc.py" > "$OUT/kpmct.log" 2>&1 || exit 4
cd "$ROOT"
python3 scripts/pmc_table.py $(find gpurun_out/kpmc1 gpurun_out/kpmc2 gpurun_out/kpmc3 gpurun_out/kpmc4 -name "*counter_collection.csv") --match gemm_kernel > gpurun_out/k12_pmc.md
cat gpurun_out/k12_pmc.md
grep gemm_kernel gpurun_out/kpmct/run_kernel_stats.csv | cut -c1-200
