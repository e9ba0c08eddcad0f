#!/bin/bash
# Throughput of the transformer BASELINE configs on one MI355X (bench/throughput.py) + a kernel profile of GPT-2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1; shift; timeout -k 10 400 python -u bench/throughput.py "$@" > gpurun_out/$name.log 2>&1 \
          || { tail -n 20 gpurun_out/$name.log; exit 3; }; tail -n 1 gpurun_out/$name.log | cut -c1-260; }
run tput_gpt2m --model gpt2-medium --batch 16 --seq 1024 --strategy dp --steps 10 --warmup 3
run tput_bertl --model bert-large --batch 32 --seq 512 --strategy dp --checkpointing all --steps 10 --warmup 3
run tput_llama1b --model llama3-1b --batch 8 --seq 2048 --strategy dp --steps 10 --warmup 3
if [ "${PROF:-1}" = 1 ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$GRAFT_REPO_ROOT/gpurun_out/prof_gpt2" -o run -- python3 "$GRAFT_REPO_ROOT/bench/throughput.py" \
     --model gpt2-medium --batch 16 --seq 1024 --strategy dp --steps 5 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof_gpt2.log" 2>&1) \
     || { tail gpurun_out/prof_gpt2.log; exit 4; }
fi
echo done
