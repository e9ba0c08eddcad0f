#!/bin/bash
# Re-entry check: GPU tests, smoke, default bench, ResNet-50-only kernel profile (batch 1024).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/gpu_tests.log" 2>&1 || { tail -n 40 "$OUT/gpu_tests.log"; exit 3; }
tail -n 1 "$OUT/gpu_tests.log"
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 4; }
tail -n 1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench.log" 2>&1 || { tail "$OUT/bench.log"; exit 5; }
tail -n 1 "$OUT/bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --model resnet50 --steps 6 --warmup 3 > "$OUT/prof.log" 2>&1 || { tail "$OUT/prof.log"; exit 6; }
tail -n 1 "$OUT/prof.log"
