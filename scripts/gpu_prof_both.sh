#!/bin/bash
# Kernel profiles of the two bench halves (ResNet-50 b1536, GPT-2 medium b64), separately.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rprof" -o run -- \
    python3 "$ROOT/bench.py" --model resnet50 --steps 5 --warmup 3 > "$OUT/rprof.log" 2>&1 || { tail "$OUT/rprof.log"; exit 3; }
tail -n 1 "$OUT/rprof.log" | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gprof" -o run -- \
    python3 "$ROOT/bench.py" --model gpt2-medium --steps 5 --warmup 3 > "$OUT/gprof.log" 2>&1 || { tail "$OUT/gprof.log"; exit 4; }
tail -n 1 "$OUT/gprof.log" | cut -c1-200
