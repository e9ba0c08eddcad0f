#!/bin/bash
# GPU A/B of the s_setprio pairs around the MFMA clusters of the attention ring kernels (knob 9)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn_prio
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench/attn_ab.py --knob 9:0:1 --rounds 7 --json $O/attn_ab_prio.json > $O/attn_ab_prio.log 2>&1 || { tail -20 $O/attn_ab_prio.log; exit 3; }
cat $O/attn_ab_prio.log
timeout -k 10 300 python -u bench.py --model gpt2-medium --steps 20 --warmup 5 > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 3; }
tail -1 $O/gpt2.log
