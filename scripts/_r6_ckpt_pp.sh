#!/bin/bash
# Round 6: training-mode leak test, GPT-2 at pipeline-rank microbatches (4 x 32 sequences under
# no_sync) per-kernel table, Llama-3 8B at 8192 tokens (planner's per-block checkpointing vs all
# blocks), the 8-GPU GPT-2 plan table at HEAD.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6b
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --model llama3-8b --seq-len 8192 --steps 3 --warmup 1 --json-out $O/llama8k_auto.json > $O/llama8k_auto.log 2>&1 || { tail -30 $O/llama8k_auto.log; exit 3; }
timeout -k 10 400 python bench.py --model llama3-8b --seq-len 8192 --steps 3 --warmup 1 --checkpointing all --json-out $O/llama8k_all.json > $O/llama8k_all.log 2>&1 || { tail -30 $O/llama8k_all.log; exit 3; }
bash scripts/gpu_profile_step.sh gpurun_out/r6b/prof_gpt2_mb32 --model gpt2-medium --steps 6 --warmup 3 --microbatches 4 || exit 3
timeout -k 10 500 python bench/plan_table.py --world 8 --only "GPT-2" --out $O/plan_tables_8gpu.md > $O/plan_table.log 2>&1 || { tail -30 $O/plan_table.log; exit 3; }
timeout -k 10 300 python bench/attn_dq_floor.py --out $O/attn_dq_floor.json > $O/attn_dq_floor.log 2>&1 || { tail -30 $O/attn_dq_floor.log; exit 3; }
echo done
