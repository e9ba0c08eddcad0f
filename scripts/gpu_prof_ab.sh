#!/bin/bash
# Kernel profiles of ResNet-50 (bench batch) with an env switch off and on: PROF_ENV=NAME.
set -u
ROOT=$(cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && pwd)
OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
NAME=${PROF_ENV:-MADNN_BN_PROLOGUE}
for v in 0 1; do
  export $NAME=$v
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_${NAME}_$v" -o run -- python3 "$ROOT/bench.py" --model resnet50 --steps 6 --warmup 4 \
      > "$OUT/prof_${NAME}_$v.log" 2>&1) || { tail -20 "$OUT/prof_${NAME}_$v.log"; exit 7; }
  tail -1 "$OUT/prof_${NAME}_$v.log"
  f=$(find "$OUT/prof_${NAME}_$v" -name "*kernel_stats.csv" | head -1)
  python3 "$ROOT/scripts/prof_summary.py" "$f" --steps 10 --top 60 --out "$OUT/prof_${NAME}_$v.md"
done
