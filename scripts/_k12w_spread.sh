#!/bin/bash
# K12W16 (the 16x16x32 form) as a weight-gradient candidate: GPU tests, A/B, re-timed Linear / 1x1 choices, bench
set -e
O=gpurun_out/k12wh
mkdir -p $O; rm -rf $O/tuning
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $O/tests.log 2>&1
tail -n 1 $O/tests.log
timeout -k 10 300 python -u bench/gemm_wgrad_ab.py --out $O/ab.json > $O/ab.log 2>&1
timeout -k 10 900 python -u scripts/record_tuning.py --out $O/tuning --keep-table --retime wgrad:linear,wgrad:conv1x1 > $O/tuning.log 2>&1
tail -n 1 $O/tuning.log
cp $O/tuning/choices_gfx950.json madnn/tuning/choices_gfx950.json
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log
python - <<'PY'
import json, collections
r=json.loads(open("gpurun_out/k12wh/bench_default.json").read().strip().splitlines()[-1])
print("resnet", r["value"], r["config"]["std_batch"]["value"], "gpt2", r["gpt2_pp"]["tokens_per_s"])
d=json.load(open("gpurun_out/k12wh/tuning/choices_gfx950.json"))["wgrad"]
print(collections.Counter((k.split(",")[0].strip("(' "), v) for k,v in d.items()))
PY
