#!/bin/bash
# Round-end rehearsal: every GPU test, smoke(), one bench.py run and a rocprofv3 kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 4; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 5; }
tail -n 1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 20 --warmup 5 \
    > gpurun_out/prof.log 2>&1 || { tail gpurun_out/prof.log; exit 6; }
tail -n 1 gpurun_out/prof.log
