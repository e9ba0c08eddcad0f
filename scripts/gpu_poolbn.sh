#!/bin/bash
# Stem BN + ReLU + max-pool fusion: tests, same-process A/B, kernel profile diff.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_gpu.py \
   -k "maxpool or pool or bottleneck or dual" > "$OUT/poolbn_tests.log" 2>&1 || { tail -40 "$OUT/poolbn_tests.log"; exit 3; }
tail -n 1 "$OUT/poolbn_tests.log"
timeout -k 10 400 python bench/resnet_flag_ab.py --flag madnn.ops:_POOL_BN --batch 1536 --windows 6 --steps 4 \
   --json-out "$OUT/ab_pool_bn.json" > "$OUT/ab_pool_bn.log" 2>&1 || { tail -20 "$OUT/ab_pool_bn.log"; exit 4; }
tail -n 1 "$OUT/ab_pool_bn.log"
PROF_ENV=MADNN_POOL_BN bash scripts/gpu_prof_ab.sh > /dev/null
