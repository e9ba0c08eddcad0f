#!/bin/bash
# GPT-2 medium DP1 (bench.py GPT-2 half, 64 sequences) kernel profile + K8 attention microbench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench/attention.py --json "$OUT/attn.json" > "$OUT/attn.log" 2>&1 || { tail "$OUT/attn.log"; exit 3; }
cat "$OUT/attn.log" | grep shape
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gprof" -o run -- \
    python3 "$ROOT/bench.py" --model gpt2-medium --steps 5 --warmup 3 > "$OUT/gprof.log" 2>&1 || { tail "$OUT/gprof.log"; exit 6; }
tail -n 1 "$OUT/gprof.log" | cut -c1-300
