#!/bin/bash
# full GPU tier, smoke, 8-GPU plan table at HEAD
set -u
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -n 3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -n 1 $O/smoke.log
timeout -k 10 500 python bench/plan_table.py --world 8 --only "GPT-2" --out $O/plan_tables_8gpu.md > $O/plan_table.log 2>&1 || { tail -30 $O/plan_table.log; exit 4; }
grep -n "choice:" $O/plan_tables_8gpu.md
