#!/bin/bash
# Round 6: GEMM / cross-entropy / model tests on the device, then the default bench and the GPT-2
# pipeline-rank microbatching (4 x 32 under no_sync) on the same box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6v
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_conv_gpu.py tests/test_conv3x3_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --json-out $O/bench_default.json > $O/bench_default.log 2>&1 || { tail -30 $O/bench_default.log; exit 3; }
timeout -k 10 300 python bench.py --model gpt2-medium --steps 10 --warmup 3 --microbatches 4 --json-out $O/gpt2_mb32x4.json > $O/gpt2_mb32x4.log 2>&1 || { tail -30 $O/gpt2_mb32x4.log; exit 3; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r6v/bench_default.json")); m = json.load(open("gpurun_out/r6v/gpt2_mb32x4.json"))
print("resnet", d["value"], d["config"]["std_batch"]["value"], "gpt2", d["gpt2_pp"]["tokens_per_s"],
      "mb32x4", m["gpt2_pp"]["tokens_per_s"], "tuning", d["config"]["tuning_timings"])
PY
