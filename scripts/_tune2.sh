#!/bin/bash
# regenerate the tuning table (incl. BERT's erf-GELU shapes), then the BERT-large steady-step table
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tune2
mkdir -p $O
timeout -k 10 900 python -u scripts/record_tuning.py --out gpurun_out/tune2/table > $O/record.log 2>&1 || { tail -30 $O/record.log; exit 3; }
tail -2 $O/record.log
bash scripts/gpu_profile_step.sh gpurun_out/tune2/prof_bert --model bert-large --steps 4 --warmup 3 || exit 3
