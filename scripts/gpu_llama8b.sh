#!/bin/bash
# Llama-3 8B, full model on ONE MI355X (288 GB): bf16 weights + fp32 masters + fp32 Adam m/v + fp32
# gradient buckets (~160 GB of state), activation checkpointing on every layer.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u bench/throughput.py --model llama3-8b --strategy dp --batch ${B:-4} --seq 2048 \
    --checkpointing ${CK:-all} --steps ${S:-4} --warmup 2 --metrics gpurun_out/llama8b_metrics.jsonl \
    > gpurun_out/tput_llama8b.log 2>&1 || { tail -n 30 gpurun_out/tput_llama8b.log; exit 3; }
tail -n 1 gpurun_out/tput_llama8b.log | cut -c1-700
