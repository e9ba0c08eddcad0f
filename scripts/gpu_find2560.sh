#!/bin/bash
# MIOpen find (exhaustive solver timing) for the ResNet-50 batch-2560 convolution shapes, with a
# heartbeat so the silent search is not mistaken for a hang; the resulting user dbs land in
# gpurun_out/miopen_db (merged into madnn/tuning/miopen afterwards).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT/miopen_db"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp madnn/tuning/miopen/* "$OUT/miopen_db/"
export MIOPEN_USER_DB_PATH="$OUT/miopen_db"
(while true; do echo "tick $(date +%s)"; ls -la "$OUT/miopen_db" | tail -2; sleep 30; done) &
TICK=$!
timeout -k 10 1000 python bench.py --model resnet50 --batch 2560 --miopen-benchmark 1 --steps 5 --warmup 2 > "$OUT/findbig.log" 2>&1
rc=$?
kill $TICK
tail -n 2 "$OUT/findbig.log"
[ $rc -ne 0 ] && exit $rc
for b in 2048 2560; do
  timeout -k 10 300 python bench.py --model resnet50 --batch $b --steps 20 --warmup 5 > "$OUT/rn_b$b.log" 2>&1 || { tail "$OUT/rn_b$b.log"; exit 5; }
  tail -n 1 "$OUT/rn_b$b.log"
done
