#!/bin/bash
# GPU check of the forward / dQ LDS-DMA attention kernels: kernel tests, then A/Bs of keys 8, 9
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn_dma
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench/attn_ab.py --knob 8:0:1 --json $O/attn_ab_fwd.json > $O/attn_ab_fwd.log 2>&1 || { tail -20 $O/attn_ab_fwd.log; exit 3; }
cat $O/attn_ab_fwd.log
timeout -k 10 300 python -u bench/attn_ab.py --knob 9:0:1 --json $O/attn_ab_dq.json > $O/attn_ab_dq.log 2>&1 || { tail -20 $O/attn_ab_dq.log; exit 3; }
cat $O/attn_ab_dq.log
