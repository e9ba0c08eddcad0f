#!/bin/bash
# rocprofv3 PMC passes (FETCH_SIZE, then WRITE_SIZE: one TCC budget each) over K11.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$ROOT/gpurun_out/pmc_k11_$c" -o run \
    -- python3 "$ROOT/bench/k11_pmc.py" > "$ROOT/gpurun_out/pmc_k11_$c.log" 2>&1 || { tail "$ROOT/gpurun_out/pmc_k11_$c.log"; exit 3; }
done
cd "$ROOT"
python3 scripts/pmc_summary.py $(find gpurun_out/pmc_k11_FETCH_SIZE -name "*counter_collection.csv" | head -n 1) \
  $(find gpurun_out/pmc_k11_WRITE_SIZE -name "*counter_collection.csv" | head -n 1) --out gpurun_out/k11_pmc.md
cat gpurun_out/k11_pmc.md
