#!/bin/bash
# Non-interactive counterpart of the reference's cifar_example/train.sh
# (which prompted for nodes / sync period / iterations and ran mpirun -npernode 1).
# One node, one process per MI355X:
#   examples/train.sh [NPROC] [SYNC_PERIOD] [ITERATIONS]
NPROC=${1:-8}
SYNC=${2:-1}
ITERS=${3:-1}
cd "$(dirname "$0")/.."
exec python -m madnn.launch --nproc "$NPROC" examples/cifar_auto_dp.py -data -usegpu -threads 1 \
    -batchSize "$SYNC" -iterations "$ITERS" -learningRate 0.001
