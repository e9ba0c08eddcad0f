#!/bin/bash
# GPU check of the inline-asm LDS-DMA switch: kernel tests, then GEMM / attention A/Bs
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/glds
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemmp_gpu.py tests/test_attention_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench/attn_ab.py --knob 7:0:1 --json $O/attn_ab.json > $O/attn_ab.log 2>&1 || { tail -20 $O/attn_ab.log; exit 3; }
timeout -k 10 400 python -u bench/gemm_ab.py --tokens 131072 --rounds 3 --json $O/gemm_ab.json > $O/gemm_ab.log 2>&1 || { tail -20 $O/gemm_ab.log; exit 3; }
timeout -k 10 400 python -u bench/gemmp_ab.py --rounds 3 --json $O/gemmp_ab.json > $O/gemmp_ab.log 2>&1 || { tail -20 $O/gemmp_ab.log; exit 3; }
