#!/bin/bash
# erf-GELU epilogues: GEMM / kernel / model tests, then the BERT-large bench (config 5) and GPT-2
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/gelu_erf
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemmp_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_gemm_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench.py --model bert-large --steps 10 --warmup 3 > $O/bert.log 2>&1 || { tail -20 $O/bert.log; exit 3; }
tail -1 $O/bert.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bert', d['value'], d['ms_per_step'], d['config']['peak_mem_gib'])"
timeout -k 10 300 python -u bench.py --model gpt2-medium --steps 10 --warmup 3 > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 3; }
tail -1 $O/gpt2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('gpt2', d['gpt2_pp']['tokens_per_s'])"
