#!/bin/bash
# ATen ops inside a ResNet-50 step (which copies / adds remain outside madnn's kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u bench/resnet_aten_ops.py --batch 256 --out gpurun_out/resnet_aten_ops.txt > gpurun_out/resnet_aten_ops.log 2>&1 || { tail -n 30 gpurun_out/resnet_aten_ops.log; exit 3; }
head -c 3000 gpurun_out/resnet_aten_ops.txt
bash scripts/gpu_r3s.sh
