#!/bin/bash
# 1-GPU bench.py records: headline (GPT-2 medium), BERT-large, Llama-3 8B
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bench_all
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/gpt2.log 2>&1 || { tail -20 $O/gpt2.log; exit 3; }
tail -1 $O/gpt2.log
timeout -k 10 400 python -u bench.py --model bert-large --steps 10 --warmup 3 > $O/bert.log 2>&1 || { tail -20 $O/bert.log; exit 3; }
tail -1 $O/bert.log
timeout -k 10 600 python -u bench.py --model llama3-8b --steps 5 --warmup 2 > $O/llama.log 2>&1 || { tail -20 $O/llama.log; exit 3; }
tail -1 $O/llama.log
