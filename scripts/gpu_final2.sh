#!/bin/bash
# Round-end rehearsal (tests, smoke, bench, profile), then the BN workgroup sweep around the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_check.sh || exit $?
for v in 2 3 6; do
  timeout -k 10 600 python bench/resnet_flag_ab.py --flag bn_tune:1 --on $v --off 4 --batch 2048 --windows 6 --steps 4 \
     --json-out gpurun_out/ab_bn_wg${v}v4.json > gpurun_out/ab_bnwg${v}v4.log 2>&1 || exit 3
  tail -1 gpurun_out/ab_bnwg${v}v4.log | cut -c1-150
done
