#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python bench/gpt2_ab.py --switch lt_res --windows 8 --steps 8 > "$OUT/ab_lt_res.log" 2>&1 || { tail -20 "$OUT/ab_lt_res.log"; exit 9; }
tail -n 1 "$OUT/ab_lt_res.log"
for b in 16 32; do
  timeout -k 10 400 python bench.py --model gpt2-medium --gpt2-batch-per-gpu $b --steps 20 --warmup 5 > "$OUT/gpt2_b$b.log" 2>&1 || { tail "$OUT/gpt2_b$b.log"; exit 5; }
  tail -n 1 "$OUT/gpt2_b$b.log"
done
