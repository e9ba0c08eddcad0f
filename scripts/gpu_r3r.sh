#!/bin/bash
# Round-3 rehearsal: every GPU test, smoke, bench (both halves), kernel profile of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export STAGES="tests smoke bench prof"
bash scripts/gpu_check.sh || exit $?
python3 scripts/prof_summary.py $(find gpurun_out/prof -name "*kernel_stats.csv") --top 40 --out gpurun_out/prof_summary.md > /dev/null || true
