#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python bench/lt_probe.py --out "$OUT/lt_probe.json" > "$OUT/lt_probe.log" 2>&1 || { tail -30 "$OUT/lt_probe.log"; exit 8; }
tail -n 60 "$OUT/lt_probe.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -n 5 "$OUT/tests.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 600 python bench.py --model gpt2-medium --steps 30 --warmup 10 > "$OUT/bench.log" 2>&1 || { tail "$OUT/bench.log"; exit 5; }
tail -n 1 "$OUT/bench.log"
