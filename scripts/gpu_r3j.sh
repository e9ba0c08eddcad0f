#!/bin/bash
# Kernel profiles of ResNet-50 alone at batch 2048 and at batch 512 (8 profiled steps each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for b in 2048 512; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rprof$b" -o run -- \
      python3 "$ROOT/bench.py" --model resnet50 --batch $b --std-batch 0 --steps 5 --warmup 3 > "$OUT/rprof$b.log" 2>&1 \
      || { tail "$OUT/rprof$b.log"; exit 3; }
  tail -n 1 "$OUT/rprof$b.log" | cut -c1-200
  python3 "$ROOT/scripts/prof_summary.py" $(find "$OUT/rprof$b" -name "*kernel_stats.csv") --steps 8 --top 45 \
      --out "$OUT/rprof$b.md" > /dev/null
done
