#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -n 5 "$OUT/tests.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python __graft_entry__.py smoke > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 4; }
tail -n 1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { tail "$OUT/bench.log"; exit 5; }
tail -n 1 "$OUT/bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 > "$OUT/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"
