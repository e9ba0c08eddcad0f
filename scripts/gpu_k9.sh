#!/bin/bash
# K9 iteration: numerics tests -> 1x1 A/B timings -> bench with and without K9.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/k9_tests.log 2>&1 || { tail -n 30 gpurun_out/k9_tests.log; exit 2; }
tail -n 1 gpurun_out/k9_tests.log
PYTHONPATH=. timeout -k 10 400 python -u bench/conv1x1_vs_gemm.py 512 --json gpurun_out/k9_ab.json > gpurun_out/k9_ab.log 2>&1 \
    || { tail -n 20 gpurun_out/k9_ab.log; exit 3; }
tail -n 1 gpurun_out/k9_ab.log
[ "${BENCH:-1}" = 1 ] || exit 0
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_k9.log 2>&1 || { tail gpurun_out/bench_k9.log; exit 4; }
tail -n 1 gpurun_out/bench_k9.log | cut -c1-200
