#!/bin/bash
# HBM bytes of madnn's kernels inside a ResNet-50 step (batch 512): one rocprofv3 pass per counter
# block (FETCH_SIZE, WRITE_SIZE), each under its own kill timeout; summary = (2xFETCH + WRITE) / time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "$OUT/rnpmc_$C" -o run -- \
    python3 "$ROOT/bench/resnet_steps.py" --batch 512 --steps 2 > "$OUT/rnpmc_$C.log" 2>&1 || { tail "$OUT/rnpmc_$C.log"; exit 3; }
done
cd "$ROOT"
python3 scripts/pmc_summary.py $(find gpurun_out/rnpmc_FETCH_SIZE -name "*counter_collection.csv") \
    $(find gpurun_out/rnpmc_WRITE_SIZE -name "*counter_collection.csv") --out gpurun_out/resnet_bn_pmc.md | head -40
