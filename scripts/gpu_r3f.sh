#!/bin/bash
# Round-3 final rehearsal: every GPU test, smoke, bench, kernel profile of the bench; then the
# downsample-gradient-in-epilogue A/B and the ATen-op census of a ResNet-50 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export STAGES="tests smoke bench prof"
bash scripts/gpu_check.sh || exit $?
python3 scripts/prof_summary.py $(find gpurun_out/prof -name "*kernel_stats.csv") --top 40 --out gpurun_out/prof_summary.md > /dev/null || true
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench/resnet_flag_ab.py --flag madnn.ops:SUB_IN_DGRAD --batch 2048 --windows 5 --steps 5 \
    > gpurun_out/ab_sub_in_dgrad.log 2>&1 || { tail -n 30 gpurun_out/ab_sub_in_dgrad.log; exit 4; }
tail -n 1 gpurun_out/ab_sub_in_dgrad.log | cut -c1-400
timeout -k 10 200 python -u bench/resnet_aten_ops.py --batch 256 --out gpurun_out/resnet_aten_ops.txt > gpurun_out/resnet_aten_ops.log 2>&1 || { tail -n 30 gpurun_out/resnet_aten_ops.log; exit 5; }
echo "all done"
