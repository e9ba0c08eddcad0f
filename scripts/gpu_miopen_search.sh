#!/bin/bash
# One 3x3 shape on MIOpen: shipped find-db (no search) vs MIOPEN_FIND_ENFORCE=SEARCH (perf-config tuning).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT/msearch_db"
export HSA_ENABLE_IPC_MODE_LEGACY=0
(while true; do echo "tick $(date +%s)"; sleep 30; done) &
TICK=$!
timeout -k 10 200 python bench/miopen_search_probe.py --cin ${CIN:-64} --hw ${HW:-56} > "$OUT/msearch_base.log" 2>&1
tail -n 1 "$OUT/msearch_base.log"
cp madnn/tuning/miopen/*.txt "$OUT/msearch_db/"
MIOPEN_USER_DB_PATH="$OUT/msearch_db" MIOPEN_FIND_ENFORCE=SEARCH timeout -k 10 ${TLIM:-700} \
  python bench/miopen_search_probe.py --cin ${CIN:-64} --hw ${HW:-56} > "$OUT/msearch_search.log" 2>&1
rc=$?
kill $TICK
tail -n 4 "$OUT/msearch_search.log"
exit $rc
