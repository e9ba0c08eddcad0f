#!/bin/bash
# K8 on the LDS-DMA three-stage ring: attention tests, K8 vs SDPA bench, GPT-2 medium bench half.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_o.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_o.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_o.log
timeout -k 10 300 python -u bench/attention.py --json gpurun_out/attn_dma.json > gpurun_out/attn_dma.log 2>&1 \
    || { tail -n 30 gpurun_out/attn_dma.log; exit 4; }
grep shape gpurun_out/attn_dma.log | cut -c1-300
timeout -k 10 400 python bench.py --model gpt2-medium --steps 20 --warmup 8 > gpurun_out/bench_gpt2_o.log 2>&1 \
    || { tail -n 30 gpurun_out/bench_gpt2_o.log; exit 5; }
tail -n 1 gpurun_out/bench_gpt2_o.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d.get('gpt2_pp',d); print({k: g.get(k) for k in ('tokens_per_s','ms_per_step','loss_last_stage')})"
