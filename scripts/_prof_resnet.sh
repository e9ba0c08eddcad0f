#!/bin/bash
# conv GPU tests, then ResNet-50 steady-step kernel tables at b2048 and b512
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_resnet
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
bash scripts/gpu_profile_step.sh gpurun_out/prof_resnet/b2048 --model resnet50 --std-batch 0 --steps 6 --warmup 3 || exit 3
bash scripts/gpu_profile_step.sh gpurun_out/prof_resnet/b512 --model resnet50 --batch 512 --std-batch 0 --steps 8 --warmup 3 || exit 3
