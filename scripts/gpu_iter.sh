#!/bin/bash
# Generic iteration: optional diagnostic script, selected GPU tests, N bench runs (+ optional A/B env).
#   DIAG=scratch/x.py TESTS="tests/a.py tests/b.py" RUNS=2 AB="MADNN_STEM=0" bash scripts/gpu_iter.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$DIAG" ]; then
  PYTHONPATH=. timeout -k 10 180 python -u $DIAG > gpurun_out/diag.log 2>&1 || { tail -n 30 gpurun_out/diag.log; exit 2; }
  grep -v "^\[madnn" gpurun_out/diag.log | tail -n 12
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/iter_tests.log 2>&1 || { tail -n 40 gpurun_out/iter_tests.log; exit 3; }
  tail -n 1 gpurun_out/iter_tests.log
fi
for r in $(seq 1 ${RUNS:-0}); do
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 8 ${BENCH_ARGS} > gpurun_out/iter_bench.log 2>&1 || { tail gpurun_out/iter_bench.log; exit 4; }
  echo "new $(tail -n 1 gpurun_out/iter_bench.log | cut -c100-160)"
  if [ -n "$AB" ]; then
    env $AB timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 8 ${BENCH_ARGS} > gpurun_out/iter_bench_ab.log 2>&1 || { tail gpurun_out/iter_bench_ab.log; exit 5; }
    echo "ab  $(tail -n 1 gpurun_out/iter_bench_ab.log | cut -c100-160)"
  fi
done
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$PROF -o run -- python bench.py --steps 15 --warmup 5 ${BENCH_ARGS} \
      > gpurun_out/$PROF.log 2>&1 || { tail gpurun_out/$PROF.log; exit 6; }
  echo prof ok
fi
