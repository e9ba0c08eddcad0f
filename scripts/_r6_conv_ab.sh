#!/bin/bash
# fresh A/Bs behind the library convolution kernels left in the ResNet-50 step: 3x3 weight-gradient
# choices re-timed (K13 vs MIOpen), stride-2 3x3 forward (K13 vs MIOpen / CK)
set -e
O=gpurun_out/r6c
mkdir -p $O; rm -rf $O/tuning
timeout -k 10 900 python -u scripts/record_tuning.py --out $O/tuning --keep-table --retime wgrad:conv3x3 --gpt2-batches "" --bert-batches "" > $O/tuning.log 2>&1
tail -n 1 $O/tuning.log
timeout -k 10 600 python -u bench/conv3x3_s2_ab.py --json $O/s2_ab.json > $O/s2_ab.log 2>&1
tail -n 8 $O/s2_ab.log
