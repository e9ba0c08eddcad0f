#!/bin/bash
# Per-shape weight-gradient candidates for ResNet-50's stride-1 convolutions at batch 2048.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench/resnet_wgrad_shapes.py --batch 2048 --json gpurun_out/wgrad_shapes_b2048.json \
    > gpurun_out/wgrad_shapes.log 2>&1 || { tail -n 30 gpurun_out/wgrad_shapes.log; exit 3; }
cat gpurun_out/wgrad_shapes.log | grep -v Warn | cut -c1-300
