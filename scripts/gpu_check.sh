#!/bin/bash
# One gpurun round: kernel tests -> smoke -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export HSA_ENABLE_IPC_MODE_LEGACY=0

stage() {  # stage <name> <timeout> <cmd...>; pytest exit 1 (test failures) is not fatal
  local name=$1 to=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name"; exit $rc; fi
  return 0
}

STAGES=${STAGES:-tests smoke bench prof}
for s in $STAGES; do
  case $s in
    tests) stage tests 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread ;;
    ktests) stage ktests 600 python -m pytest tests/test_kernels_gpu.py -q ;;
    smoke) stage smoke 400 python __graft_entry__.py smoke ;;
    bench) stage bench 600 python bench.py --steps 30 --warmup 10 ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 5 > "$OUT/prof.log" 2>&1)
      rc=$?; echo "== prof rc=$rc"; tail -n 5 "$OUT/prof.log"; [ $rc -ne 0 ] && exit $rc ;;
    *) stage "$s" 900 bash -c "$s" ;;
  esac
done
echo "== all stages done"
