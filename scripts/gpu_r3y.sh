#!/bin/bash
# K6f v2 (one exp per element): tests, GPT-2 A/B; ResNet-50 b2048 steady-state kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_y.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_y.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_y.log
timeout -k 10 400 python -u bench/gpt2_ab.py --batch 64 --switch xent --windows 6 --steps 6 \
    > gpurun_out/ab_xent2.log 2>&1 || { tail -n 30 gpurun_out/ab_xent2.log; exit 4; }
tail -n 1 gpurun_out/ab_xent2.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/rtrace4" -o run -- \
    python3 "$ROOT/bench.py" --model resnet50 --std-batch 0 --steps 5 --warmup 3 > "$ROOT/gpurun_out/rtrace4.log" 2>&1 || { tail "$ROOT/gpurun_out/rtrace4.log"; exit 5; }
cd "$ROOT"
python3 scripts/trace_steps.py $(find gpurun_out/rtrace4 -name "*kernel_trace.csv") --last 4 --top 70 --out gpurun_out/resnet_steady4.md > gpurun_out/resnet_steady4.txt
