#!/bin/bash
# K12W filler-spread A/B: correctness of each variant then V=1 (pair statements) vs V=2 (single pieces over two phases)
set -e
mkdir -p gpurun_out/k12ws
for V in 1 2; do
MADNN_K12W_V=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k wgrad > gpurun_out/k12ws/tests_v$V.log 2>&1
done
for R in a b; do for V in 1 2; do
MADNN_K12W_V=$V timeout -k 10 300 python -u bench/gemm_wgrad_ab.py --out gpurun_out/k12ws/v$V$R.json > gpurun_out/k12ws/v$V$R.log 2>&1
done; done
tail -1 gpurun_out/k12ws/tests_v1.log gpurun_out/k12ws/tests_v2.log
python - <<'PY'
import json
for v in ("v1a","v2a","v1b","v2b"):
    rows=json.load(open(f"gpurun_out/k12ws/{v}.json"))
    print(v, " ".join(f"{r['shape'].replace(' ','_')}:{r['k12w_us']:.0f}" for r in rows))
PY
