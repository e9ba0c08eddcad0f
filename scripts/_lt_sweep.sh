#!/bin/bash
# hipBLASLt ranked-candidate sweep on the GPT-2 b128 Linear shapes
set -e
mkdir -p gpurun_out/lt_sweep
timeout -k 10 600 python -u bench/lt_algo_sweep.py > gpurun_out/lt_sweep/sweep.jsonl 2> gpurun_out/lt_sweep/err.log
cat gpurun_out/lt_sweep/sweep.jsonl
