#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_gpu.py tests/test_conv3x3_gpu.py \
   -k "dgrad_epilogue or bottleneck or conv3x3" > "$OUT/bnepi_tests.log" 2>&1 || { tail -40 "$OUT/bnepi_tests.log"; exit 3; }
tail -n 1 "$OUT/bnepi_tests.log"
timeout -k 10 500 python bench/resnet_flag_ab.py --flag madnn.ops:_BN_DGRAD_EPI --batch 2048 --windows 6 --steps 4 \
   --json-out "$OUT/ab_bn_dgrad_epi.json" > "$OUT/ab_bn_dgrad_epi.log" 2>&1 || { tail -20 "$OUT/ab_bn_dgrad_epi.log"; exit 4; }
tail -n 1 "$OUT/ab_bn_dgrad_epi.log"
