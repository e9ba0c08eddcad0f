set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/prof" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 5 > "$ROOT/gpurun_out/prof.log" 2>&1) || { tail -20 gpurun_out/prof.log; exit 7; }
tail -1 gpurun_out/prof.log
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py "$f" --steps 25 --top 70 --out gpurun_out/prof_summary.md
