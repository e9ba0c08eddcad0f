#!/bin/bash
# PMC passes over the K8 attention kernels at the GPT-2 medium shape (bench/attn_prof.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export ATTN_SHAPE=${ATTN_SHAPE:-16,1024,16,16,64} ATTN_ITERS=2
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_MFMA,SQ_INSTS_LDS,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT
P2=SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_INSTS_VALU_TRANS_F32,SQ_ACTIVE_INST_ANY,SQ_WAIT_ANY,SQ_INSTS_SALU,SQ_WAVES
cd /tmp && export TMPDIR=/tmp
i=0
for P in $P1 $P2; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${P//,/ } --output-format csv -d "$OUT/apmc$i" -o run -- \
    python3 "$ROOT/bench/attn_prof.py" > "$OUT/apmc$i.log" 2>&1 || { tail "$OUT/apmc$i.log"; exit 3; }
done
cd "$ROOT"
python3 scripts/pmc_table.py $(find gpurun_out/apmc1 gpurun_out/apmc2 -name "*counter_collection.csv") --match attn \
  > gpurun_out/attn_pmc.md
cat gpurun_out/attn_pmc.md
