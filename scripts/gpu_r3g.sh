#!/bin/bash
# final-tree bench (both halves), one run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export STAGES="smoke bench"
bash scripts/gpu_check.sh || exit $?
