#!/bin/bash
# model GPU tests, then the GPT-2 medium b128 steady-step kernel table
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_gpt2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
bash scripts/gpu_profile_step.sh gpurun_out/prof_gpt2/step --model gpt2-medium --steps 6 --warmup 3
