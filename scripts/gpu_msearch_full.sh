#!/bin/bash
# MIOpen perf-config SEARCH over every ResNet-50 convolution that still runs on MIOpen (batch
# 1536), into a copy of the shipped db; then find-off bench runs with the shipped vs searched db.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; DB="$OUT/msearch_full"; mkdir -p "$DB"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp madnn/tuning/miopen/*.txt "$DB/"
(while true; do echo "tick $(date +%s) $(wc -l < $DB/*.udb.txt)"; sleep 30; done) &
TICK=$!
MIOPEN_USER_DB_PATH="$DB" MIOPEN_FIND_ENFORCE=SEARCH timeout -k 10 ${TLIM:-780} \
  python bench.py --model resnet50 --miopen-benchmark 1 --steps 3 --warmup 2 > "$OUT/msearch_full.log" 2>&1
echo "search rc=$?"
kill $TICK
tail -n 1 "$OUT/msearch_full.log" | cut -c1-200
timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 > "$OUT/ms_shipped.log" 2>&1 || exit 5
tail -n 1 "$OUT/ms_shipped.log" | cut -c1-200
MIOPEN_USER_DB_PATH="$DB" timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 > "$OUT/ms_searched.log" 2>&1 || exit 6
tail -n 1 "$OUT/ms_searched.log" | cut -c1-200
