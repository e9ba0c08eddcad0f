#!/bin/bash
# TunableOp A/B: tune every GEMM shape of a workload (hipBLASLt + rocBLAS solutions), then re-run
# reading the tuned file only, against the untuned baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tunableop
export HSA_ENABLE_IPC_MODE_LEGACY=0
G="--model gpt2-medium --batch 16 --seq 1024 --strategy dp"
R="--steps 20 --warmup 8"
tput() { local name=$1; shift; timeout -k 10 400 python -u bench/throughput.py "$@" > gpurun_out/$name.log 2>&1 \
          || { tail -n 20 gpurun_out/$name.log; exit 3; }; echo "$name $(tail -n 1 gpurun_out/$name.log | cut -c1-160)"; }
bench() { local name=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/$name.log 2>&1 \
          || { tail -n 20 gpurun_out/$name.log; exit 4; }; echo "$name $(tail -n 1 gpurun_out/$name.log | cut -c100-150)"; }
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop/tunableop_results%d.csv
tput gpt2_base $G --steps 10 --warmup 3
# tuning pass (verbose output keeps the log growing while it searches)
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
  tput gpt2_tune $G --steps 2 --warmup 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 tput gpt2_tuned $G --steps 10 --warmup 3
bench rn_base $R
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 bench rn_tune --steps 2 --warmup 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 bench rn_tuned $R
bench rn_base2 $R
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 bench rn_tuned2 $R
wc -l gpurun_out/tunableop/*.csv
