#!/bin/bash
# D = 128 attention at 2 waves per SIMD: attention / model / glue tests, Llama-3 8B bench
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn128
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_models_gpu.py tests/test_glue_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --model llama3-8b --steps 5 --warmup 2 > $O/llama.log 2>&1 || { tail -20 $O/llama.log; exit 3; }
tail -1 $O/llama.log
