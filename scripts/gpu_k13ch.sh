#!/bin/bash
# K13 chunk width 32 vs 64: correctness (both widths), then the A/B against MIOpen.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 32 64; do
  MADNN_K13_CH=$v timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 120 \
     --timeout-method thread -k "conv3x3 or k13" > $OUT/k13ch_tests$v.log 2>&1; rc=$?; echo "CH=$v"; tail -n 3 $OUT/k13ch_tests$v.log; [ $rc -ne 0 ] && exit $rc
done
for v in 64 32; do MADNN_K13_CH=$v timeout -k 10 200 python bench/conv3x3_ab.py --rounds 3 > $OUT/k13ch$v.log 2>&1 || exit 3
  echo "CH=$v"; grep '"C"' $OUT/k13ch$v.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['C'], 'fwd', r['fwd_k13_us'], 'dgrad', r['dgrad_k13_us'], 'miopen', r['fwd_miopen_us'], r['dgrad_miopen_us'])"; done
