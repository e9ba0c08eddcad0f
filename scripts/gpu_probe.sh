#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"
timeout -k 10 300 python bench/lt_probe.py --out "$OUT/lt_probe.json" > "$OUT/lt_probe.log" 2>&1 || { tail -30 "$OUT/lt_probe.log"; exit 8; }
tail -n 40 "$OUT/lt_probe.log"
