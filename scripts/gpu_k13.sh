#!/bin/bash
# K13 3x3 conv: GPU correctness tests, then the A/B against MIOpen on the ResNet-50 shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/k13_tests.log 2>&1; rc=$?; tail -n 30 $OUT/k13_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench/conv3x3_ab.py --json $OUT/k13_ab.json > $OUT/k13_ab.log 2>&1; rc=$?
tail -n 6 $OUT/k13_ab.log; exit $rc
