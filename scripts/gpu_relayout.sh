#!/bin/bash
# Streaming bucket re-layout: engine GPU tests, then Llama-3 8B on one GPU (peak HBM).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread \
   > gpurun_out/relayout_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/relayout_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench/throughput.py --model llama3-8b --strategy dp --batch 4 --seq 2048 --checkpointing all \
   --steps 4 --warmup 2 > gpurun_out/r2_tput_llama8b.log 2>&1 || { tail -n 20 gpurun_out/r2_tput_llama8b.log; exit 3; }
tail -n 1 gpurun_out/r2_tput_llama8b.log | cut -c1-300
