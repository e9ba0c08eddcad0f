#!/bin/bash
# K12 with the conflict-free 16x16x32 row image: GEMM tests, per-shape A/B (M16 vs M32 vs hipBLASLt), PMC pass 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_h.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_h.log; exit 3; }
tail -n 1 gpurun_out/gpu_tests_h.log
timeout -k 10 400 python -u bench/gemm_ab.py --json gpurun_out/gemm_ab_h.json > gpurun_out/gemm_ab_h.log 2>&1 \
    || { tail -n 30 gpurun_out/gemm_ab_h.log; exit 4; }
python3 -c "
import json
for r in json.load(open('gpurun_out/gemm_ab_h.json')):
    print(r['shape'], {k: v for k, v in r.items() if k.endswith('_us')})"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_MFMA \
    --output-format csv -d "$ROOT/gpurun_out/hpmc1" -o run -- python3 "$ROOT/bench/k12_pmc.py" > "$ROOT/gpurun_out/hpmc1.log" 2>&1 || exit 5
cd "$ROOT"
python3 scripts/pmc_table.py $(find gpurun_out/hpmc1 -name "*counter_collection.csv") --match gemm_kernel
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_h_attn.log 2>&1 || { tail -n 40 gpurun_out/gpu_tests_h_attn.log; exit 6; }
tail -n 1 gpurun_out/gpu_tests_h_attn.log
timeout -k 10 300 python -u bench/attention.py --native madnn_attn_tune:0:1:0 --json gpurun_out/attn_ab_v2.json \
    > gpurun_out/attn_ab_v2.log 2>&1 || { tail -n 30 gpurun_out/attn_ab_v2.log; exit 7; }
cat gpurun_out/attn_ab_v2.log | grep shape | cut -c1-400
