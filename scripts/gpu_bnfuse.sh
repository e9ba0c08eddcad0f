#!/bin/bash
# Round-2 BN fusions: dual downsample BN (K5 RAFF) and bn2 -> conv3 K9 prologue: tests, then
# same-process A/B of each switch on ResNet-50 at the bench batch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_conv_gpu.py \
   -k "dual or prologue or batchnorm or bottleneck or three_passes" > "$OUT/bnfuse_tests.log" 2>&1 || { tail -40 "$OUT/bnfuse_tests.log"; exit 3; }
tail -n 2 "$OUT/bnfuse_tests.log"
timeout -k 10 400 python bench/resnet_flag_ab.py --flag madnn.models.resnet:_DUAL_BN --batch 1536 --windows 6 --steps 4 \
   --json-out "$OUT/ab_dual_bn.json" > "$OUT/ab_dual_bn.log" 2>&1 || { tail -20 "$OUT/ab_dual_bn.log"; exit 4; }
tail -n 1 "$OUT/ab_dual_bn.log"
timeout -k 10 400 python bench/resnet_flag_ab.py --flag madnn.ops:_BN_PROLOGUE --batch 1536 --windows 6 --steps 4 \
   --json-out "$OUT/ab_bn_prologue.json" > "$OUT/ab_bn_prologue.log" 2>&1 || { tail -20 "$OUT/ab_bn_prologue.log"; exit 5; }
tail -n 1 "$OUT/ab_bn_prologue.log"
