#!/bin/bash
# Deferred ReLU mask (bn3 -> K9 dgrad): conv tests + ResNet A/B; planner test in a fresh process;
# GPT-2 kernel trace to confirm the bias-grad passes the column sums replaced.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_planner_gpu.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_u.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_u.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_u.log
timeout -k 10 600 python bench/resnet_flag_ab.py --flag madnn.ops:DEFER_RES_MASK --on true --off false --batch 2048 \
   --windows 6 --steps 4 --json-out gpurun_out/ab_defer_mask_b2048.json > gpurun_out/ab_defer_mask.log 2>&1 \
   || { tail -n 30 gpurun_out/ab_defer_mask.log; exit 4; }
tail -n 1 gpurun_out/ab_defer_mask.log | cut -c1-260
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/gtrace" -o run -- \
    python3 "$ROOT/bench.py" --model gpt2-medium --steps 4 --warmup 3 > "$ROOT/gpurun_out/gtrace.log" 2>&1 || { tail "$ROOT/gpurun_out/gtrace.log"; exit 5; }
cd "$ROOT"
python3 scripts/trace_steps.py $(find gpurun_out/gtrace -name "*kernel_trace.csv") --last 3 --top 30 --out gpurun_out/gpt2_steady.md | head -40
