#!/bin/bash
# Round-3 first check: every GPU test, smoke(), one default bench.py run (2048 + std 512 + GPT-2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 4; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 10 > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 5; }
tail -n 1 gpurun_out/bench.log
