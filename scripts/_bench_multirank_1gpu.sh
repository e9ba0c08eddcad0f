#!/bin/bash
# bench.py's N = 2 and N = 4 code paths (ResNet-50 DP + GPT-2 pipeline) with every rank on this one
# GPU over gloo (RCCL refuses two ranks on one device): small batches, a few steps -- a rehearsal of
# the driver's multi-GPU run, not a performance number
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/multirank
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for N in 2 4; do
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29500 + N)) bench.py --gpus $N --steps 3 --warmup 2 --backend gloo --batch 256 \
      --std-batch 0 --gpt2-batch-per-gpu 16 > $O/n$N.log 2>&1 || { tail -30 $O/n$N.log; exit 3; }
  grep '^{' $O/n$N.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gpt2_pp']; print('N', d['n_gpus'], d['value'], d['config']['parallelism'], g.get('parallelism'), g.get('tokens_per_s'), g.get('schedule'), g.get('error'))"
done
