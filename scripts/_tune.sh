#!/bin/bash
# conv tests, then regenerate the shipped start-up tuning table (scripts/record_tuning.py)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tune
mkdir -p $O
timeout -k 10 900 python -u scripts/record_tuning.py --out gpurun_out/tune/table > $O/record.log 2>&1 || { tail -30 $O/record.log; exit 3; }
tail -3 $O/record.log
