#!/bin/bash
# K12 GEMM: correctness tests, then the interleaved A/B against hipBLASLt on the GPT-2 shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -v --timeout 120 --timeout-method thread \
    > $OUT/k12_tests.log 2>&1; rc=$?; tail -n 25 $OUT/k12_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench/gemm_ab.py --json $OUT/k12_ab.json > $OUT/k12_ab.log 2>&1; rc=$?
cat $OUT/k12_ab.log | tail -n 12; exit $rc
