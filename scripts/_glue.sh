#!/bin/bash
# K14 / K15 tests, transformer model tests, then the Llama-3 8B bench (config 4)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/glue
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_glue_gpu.py tests/test_attention_gpu.py tests/test_models_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 600 python -u bench.py --model llama3-8b --steps 5 --warmup 2 > $O/llama.log 2>&1 || { tail -20 $O/llama.log; exit 3; }
tail -1 $O/llama.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['peak_mem_gib'], d['config']['checkpointed_layers'])"
