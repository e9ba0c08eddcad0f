#!/bin/bash
# Full GPU test tier, then an optional ResNet flag A/B (AB_FLAG / AB_ON / AB_OFF / AB_NAME).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?
tail -n 3 "$OUT/tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${AB_FLAG:-}" ]; then
  timeout -k 10 400 python bench/resnet_flag_ab.py --flag "$AB_FLAG" --on "$AB_ON" --off "$AB_OFF" --batch 1536 --windows 6 \
     --steps 4 --json-out "$OUT/ab_${AB_NAME}.json" > "$OUT/ab_${AB_NAME}.log" 2>&1 || { tail -20 "$OUT/ab_${AB_NAME}.log"; exit 4; }
  tail -n 1 "$OUT/ab_${AB_NAME}.log"
fi
exit $rc
