#!/bin/bash
# HEAD validation: full GPU tier, smoke, default bench, GPT-2 b128 steady-step kernel table
set -u
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -n 3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -n 1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log || { tail -20 $O/bench_default.log; exit 4; }
python - <<'PY'
import json
r=json.loads(open("gpurun_out/r6f/bench_default.json").read().strip().splitlines()[-1])
print("resnet", r["value"], r["config"]["std_batch"]["value"], "gpt2", r["gpt2_pp"]["tokens_per_s"])
PY
bash scripts/gpu_profile_step.sh gpurun_out/r6f/prof_gpt2 --model gpt2-medium --steps 6 --warmup 3 > $O/prof.log 2>&1 || exit 5
head -8 gpurun_out/r6f/prof_gpt2/steps.md
