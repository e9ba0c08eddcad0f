set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for d in 0 2 3 4; do MADNN_K13_DBG=$d timeout -k 10 200 python bench/conv3x3_ab.py --rounds 3 > gpurun_out/k13dbg$d.log 2>&1 || exit 3; echo "dbg=$d"; grep '"C"' gpurun_out/k13dbg$d.log | python3 -c "
import json,sys
for l in sys.stdin:
    r=json.loads(l); print(r['C'], 'fwd', r['fwd_k13_us'], 'dgrad', r['dgrad_k13_us'])"; done
