#!/bin/bash
# GPU check after a kernel change: every kernel test file, then the GPT-2 bench step
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/kcheck
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_gpu.py tests/test_gemmp_gpu.py tests/test_attention_gpu.py tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['std_batch']['value'], d['gpt2_pp']['tokens_per_s'])"
