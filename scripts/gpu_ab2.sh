#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k gelu_fwd --timeout 120 > "$OUT/gelu_test.log" 2>&1 || { tail -20 "$OUT/gelu_test.log"; exit 3; }
tail -n 1 "$OUT/gelu_test.log"
timeout -k 10 400 python bench/gpt2_ab.py --switch gelu --batch 32 --windows 8 --steps 6 > "$OUT/ab_gelu.log" 2>&1 || { tail -20 "$OUT/ab_gelu.log"; exit 9; }
tail -n 1 "$OUT/ab_gelu.log"
timeout -k 10 400 python bench/resnet_ab.py --a bucket_mb=64 --b bucket_mb=0 --windows 8 --steps 6 > "$OUT/ab_resnet_bucket.log" 2>&1 || { tail -20 "$OUT/ab_resnet_bucket.log"; exit 9; }
tail -n 1 "$OUT/ab_resnet_bucket.log"
