#!/bin/bash
# Rehearsal (tests, smoke, default bench) + GPT-2 sequences-per-GPU sweep above 64.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
STAGES="tests smoke bench" bash scripts/gpu_check.sh || exit $?
for b in 96 128; do
  timeout -k 10 400 python bench.py --model gpt2-medium --gpt2-batch-per-gpu $b --steps 10 --warmup 4 > "$OUT/gpt2_b$b.log" 2>&1 || { tail "$OUT/gpt2_b$b.log"; exit 5; }
  tail -n 1 "$OUT/gpt2_b$b.log" | cut -c1-200; grep -o '"tokens_per_s": [0-9.]*' "$OUT/gpt2_b$b.log"; grep -o '"peak_mem_gib": [0-9.]*' "$OUT/gpt2_b$b.log"
done
