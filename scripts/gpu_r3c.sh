#!/bin/bash
# Planner accuracy after the model-input fix: the GPU test + the 4-case table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u bench/plan_accuracy.py --json-out gpurun_out/plan_acc.json > gpurun_out/plan_acc.log 2>&1 \
    || { tail -n 40 gpurun_out/plan_acc.log; exit 4; }
grep '^{' gpurun_out/plan_acc.log
timeout -k 10 400 python -u -m pytest tests/test_planner_gpu.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_c.log 2>&1 || { tail -n 60 gpurun_out/gpu_tests_c.log; exit 3; }
tail -n 3 gpurun_out/gpu_tests_c.log
