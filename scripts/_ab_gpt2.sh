#!/bin/bash
# A/B: GPT-2 medium bench step with the GELU epilogues on hipBLASLt+K11 (lt) vs auto (K12P when faster)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_gpt2
mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemmp_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
for rep in 1 2; do
  for arm in lt auto; do
    MADNN_GELU_FWD=$arm MADNN_DGELU=$arm timeout -k 10 300 python -u bench.py --model gpt2-medium --steps 10 --warmup 3 > $O/${arm}_$rep.log 2>&1 || { tail -20 $O/${arm}_$rep.log; exit 3; }
    grep -o '"tokens_per_s": [0-9.]*' $O/${arm}_$rep.log | head -1
  done
done
