#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "walk_variants or batchnorm" \
   > "$OUT/bn_walk.log" 2>&1 || { tail -30 "$OUT/bn_walk.log"; exit 3; }
tail -n 1 "$OUT/bn_walk.log"
timeout -k 10 500 python bench/resnet_flag_ab.py --flag bn_tune:3 --on 1 --off 0 --batch 2048 --windows 6 --steps 4 \
   --json-out "$OUT/ab_bn_unroll.json" > "$OUT/ab_bn_unroll.log" 2>&1 || { tail -20 "$OUT/ab_bn_unroll.log"; exit 4; }
tail -n 1 "$OUT/ab_bn_unroll.log"
