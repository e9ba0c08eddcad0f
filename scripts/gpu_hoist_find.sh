#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "batchnorm or maxpool" \
   > "$OUT/bn_kernels.log" 2>&1 || { tail -30 "$OUT/bn_kernels.log"; exit 3; }
tail -n 1 "$OUT/bn_kernels.log"
timeout -k 10 400 python bench/resnet_flag_ab.py --flag bn_tune:2 --on 1 --off 0 --batch 1536 --windows 6 --steps 4 \
   --json-out "$OUT/ab_bn_hoist.json" > "$OUT/ab_bn_hoist.log" 2>&1 || { tail -20 "$OUT/ab_bn_hoist.log"; exit 4; }
tail -n 1 "$OUT/ab_bn_hoist.log"
bash scripts/gpu_find2048.sh
