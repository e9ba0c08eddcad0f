#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 4 8 64; do
  timeout -k 10 400 python bench.py --model gpt2-medium --gpt2-batch-per-gpu $b --steps 12 --warmup 4 > "$OUT/gpt2_b$b.log" 2>&1 || { tail "$OUT/gpt2_b$b.log"; exit 5; }
  tail -n 1 "$OUT/gpt2_b$b.log"
done
