#!/bin/bash
# dq column sums through LDS: attention tests, GPT-2 attn-colsum A/B, steady-state GPT-2 trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_v.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_v.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_v.log
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch attn_colsum --windows 6 --steps 6 \
    > gpurun_out/ab_attn_colsum2.log 2>&1 || { tail -n 30 gpurun_out/ab_attn_colsum2.log; exit 4; }
tail -n 1 gpurun_out/ab_attn_colsum2.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/gtrace2" -o run -- \
    python3 "$ROOT/bench.py" --model gpt2-medium --steps 4 --warmup 3 > "$ROOT/gpurun_out/gtrace2.log" 2>&1 || { tail "$ROOT/gpurun_out/gtrace2.log"; exit 5; }
cd "$ROOT"
python3 scripts/trace_steps.py $(find gpurun_out/gtrace2 -name "*kernel_trace.csv") --last 3 --top 12 --out gpurun_out/gpt2_steady2.md > gpurun_out/gpt2_steady2.txt
