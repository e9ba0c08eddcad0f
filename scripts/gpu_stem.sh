#!/bin/bash
# K10 iteration: stem numerics tests -> bench with and without K10 -> kernel-stats profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_stem_gpu.py -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/k10_tests.log 2>&1 || { tail -n 40 gpurun_out/k10_tests.log; exit 2; }
tail -n 1 gpurun_out/k10_tests.log
[ "${BENCH:-1}" = 1 ] || exit 0
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_k10.log 2>&1 || { tail gpurun_out/bench_k10.log; exit 4; }
  echo "k10 $(tail -n 1 gpurun_out/bench_k10.log | cut -c1-120)"
  MADNN_STEM=0 timeout -k 10 300 python bench.py --steps 20 --warmup 8 > gpurun_out/bench_nok10.log 2>&1 || { tail gpurun_out/bench_nok10.log; exit 5; }
  echo "miopen $(tail -n 1 gpurun_out/bench_nok10.log | cut -c1-120)"
done
[ "${PROF:-1}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k10 -o run -- python bench.py --steps 15 --warmup 5 \
    > gpurun_out/prof_k10.log 2>&1 || { tail gpurun_out/prof_k10.log; exit 6; }
echo prof ok
