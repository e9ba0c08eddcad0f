#!/bin/bash
# Round-3 refresh of the transformer BASELINE configs on one MI355X (bench/throughput.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; timeout -k 10 600 python -u bench/throughput.py "$@" > gpurun_out/$name.log 2>&1 \
          || { tail -n 20 gpurun_out/$name.log; exit 3; }; tail -n 1 gpurun_out/$name.log | cut -c1-300; }
run r3_tput_bertl --model bert-large --batch 64 --seq 512 --strategy dp --checkpointing all --steps 8 --warmup 3
run r3_tput_llama1b --model llama3-1b --batch 16 --seq 2048 --strategy dp --steps 8 --warmup 3
run r3_tput_llama8b --model llama3-8b --strategy dp --batch 4 --seq 2048 --checkpointing all --steps 4 --warmup 2
echo done
