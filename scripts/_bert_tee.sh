#!/bin/bash
# BERT attention-residual fold (ops.linear_tee): GEMM / model tests, BERT steady-step table and bench
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bert_tee
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemmp_gpu.py tests/test_models_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
bash scripts/gpu_profile_step.sh gpurun_out/bert_tee/prof --model bert-large --steps 4 --warmup 3 || exit 3
timeout -k 10 400 python -u bench.py --model bert-large --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
tail -1 $O/bench.log | cut -c1-250
