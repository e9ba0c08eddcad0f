#!/bin/bash
# GPU A/B of the attention kernels' occupancy targets (knob 9: bit 0 register-staged forward / dQ at
# 2 waves per SIMD, bit 1 forward ring at 3)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/attn_occ
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_attention_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
for k in 9:0:1; do
  timeout -k 10 300 python -u bench/attn_ab.py --knob $k --rounds 7 --json $O/ab_${k//:/_}.json > $O/ab_${k//:/_}.log 2>&1 || { tail -20 $O/ab_${k//:/_}.log; exit 3; }
  cat $O/ab_${k//:/_}.log
done
