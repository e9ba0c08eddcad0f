#!/bin/bash
# one-pass cross entropy (K6f) + delta in the dQ prologue: tests, GPT-2 A/Bs, steady-state GPT-2 trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_attention_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_w.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_w.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_w.log
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch xent --windows 6 --steps 6 \
    > gpurun_out/ab_xent.log 2>&1 || { tail -n 30 gpurun_out/ab_xent.log; exit 4; }
tail -n 1 gpurun_out/ab_xent.log | cut -c1-300
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch native --native madnn_attn_tune:1:1:0 --windows 6 --steps 6 \
    > gpurun_out/ab_dq_delta.log 2>&1 || { tail -n 30 gpurun_out/ab_dq_delta.log; exit 6; }
tail -n 1 gpurun_out/ab_dq_delta.log | cut -c1-300
timeout -k 10 400 python -u bench/resnet_flag_ab.py --flag madnn.ops:BN_SUM_IN_DGRAD --batch 2048 --windows 5 --steps 5 \
    > gpurun_out/ab_bn_sum.log 2>&1 || { tail -n 30 gpurun_out/ab_bn_sum.log; exit 7; }
tail -n 1 gpurun_out/ab_bn_sum.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/gtrace3" -o run -- \
    python3 "$ROOT/bench.py" --model gpt2-medium --steps 4 --warmup 3 > "$ROOT/gpurun_out/gtrace3.log" 2>&1 || { tail "$ROOT/gpurun_out/gtrace3.log"; exit 5; }
cd "$ROOT"
python3 scripts/trace_steps.py $(find gpurun_out/gtrace3 -name "*kernel_trace.csv") --last 3 --top 40 --out gpurun_out/gpt2_steady3.md > gpurun_out/gpt2_steady3.txt
