#!/bin/bash
# Steady-state kernel profile of the bench step: rocprofv3 kernel trace of bench.py, then the
# per-kernel table of the last steps (scripts/trace_steps.py).
#   bash scripts/gpu_profile_step.sh <out dir> <bench.py args...>
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/$1"; shift
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv \
    -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" "$@" > "$OUT/bench.log" 2>&1) || { tail -20 "$OUT/bench.log"; exit 3; }
CSV=$(python3 -c "import glob,sys; f=sorted(glob.glob(sys.argv[1]+'/**/*kernel_trace.csv', recursive=True)); print(f[0] if f else '')" "$OUT/trace")
[ -n "$CSV" ] || { echo "no kernel trace under $OUT/trace"; exit 3; }
python3 "$ROOT/scripts/trace_steps.py" "$CSV" --last 4 --top 40 --out "$OUT/steps.md" && head -3 "$OUT/steps.md"
