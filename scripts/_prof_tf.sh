#!/bin/bash
# steady-step kernel tables of the transformer configs: Llama-3 8B (config 4) and BERT-large (config 5)
set -u
bash scripts/gpu_profile_step.sh gpurun_out/prof_llama2 --model llama3-8b --steps 3 --warmup 2 || exit 3
bash scripts/gpu_profile_step.sh gpurun_out/prof_bert --model bert-large --steps 4 --warmup 3 || exit 3
