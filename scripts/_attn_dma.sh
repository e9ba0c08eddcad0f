#!/bin/bash
# GPU check of the attention kernels: kernel / model tests, then the forward DMA A/B (absolute times)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn_pre2
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_models_gpu.py tests/test_gemmp_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench/attn_ab.py --knob 8:0:1 --json $O/attn_ab_fwd.json > $O/attn_ab_fwd.log 2>&1 || { tail -20 $O/attn_ab_fwd.log; exit 3; }
cat $O/attn_ab_fwd.log
timeout -k 10 300 python -u bench/attn_ab.py --knob 7:0:1 --json $O/attn_ab_dkdv.json > $O/attn_ab_dkdv.log 2>&1 || { tail -20 $O/attn_ab_dkdv.log; exit 3; }
cat $O/attn_ab_dkdv.log
timeout -k 10 300 python -u bench.py --model gpt2-medium --steps 10 --warmup 3 > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 3; }
tail -1 $O/gpt2.log | grep -o '"tokens_per_s": [0-9.]*'
