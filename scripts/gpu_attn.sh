#!/bin/bash
# K8 attention: GPU correctness tests, then the SDPA comparison bench (3 shapes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/attn_tests.log 2>&1; rc=$?; tail -n 3 $OUT/attn_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench/attention.py --json $OUT/attn.json > $OUT/attn.log 2>&1; rc=$?
grep shape $OUT/attn.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['shape'], 'fwd', r['k8_fwd_ms'], r['k8_fwd_tflops'], 'bwd', r['k8_bwd_ms'], r['k8_bwd_tflops'])"
exit $rc
