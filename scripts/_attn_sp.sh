#!/bin/bash
# software-pipelined D = 64 forward (knob 9): attention tests, then the A/B
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn_sp
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench/attn_ab.py --knob 9:0:1 --rounds 7 --json $O/ab.json > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 3; }
cat $O/ab.log
