#!/bin/bash
# K12W (pinned schedule): GPU tests of the GEMM/conv paths, re-time the Linear / 1x1 weight-gradient choices, bench with them
set -e
mkdir -p gpurun_out/r6t; rm -rf gpurun_out/r6t/tuning
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemmp_gpu.py tests/test_models_gpu.py > gpurun_out/r6t/tests.log 2>&1
tail -n1 gpurun_out/r6t/tests.log
timeout -k 10 900 python -u scripts/record_tuning.py --out gpurun_out/r6t/tuning --keep-table --retime dgrad:* > gpurun_out/r6t/tuning.log 2>&1
tail -n1 gpurun_out/r6t/tuning.log
cp gpurun_out/r6t/tuning/choices_gfx950.json madnn/tuning/choices_gfx950.json
timeout -k 10 600 python -u bench.py > gpurun_out/r6t/bench_default.json 2> gpurun_out/r6t/bench_default.log
python - <<'PY'
import json
r=json.loads(open("gpurun_out/r6t/bench_default.json").read().strip().splitlines()[-1])
print("resnet", r["value"], r["config"]["std_batch"]["value"], "gpt2", r["gpt2_pp"]["tokens_per_s"], "tuning", r["config"].get("tuning_timings"))
PY
