#!/usr/bin/env python3
"""K3 LayerNorm forward / backward at the GPT-2 medium (131072 x 1024) and BERT-large (65536 x 1024)
shapes, bf16, against the launch-grid knobs (madnn_norm_tune 0 / 1): time and achieved bandwidth
(forward 4 B, backward 6 B per element).  python bench/norm_probe.py"""
import ctypes, statistics, torch, sys, os, json
sys.path.insert(0, os.getcwd())
from madnn import ops
assert ops.load_kernels()
tune = ctypes.CDLL(str(ops.kernels_path())).madnn_norm_tune
def timeit(fn, iters=20):
    for _ in range(3): fn()
    ts=[]
    for _ in range(iters):
        s,e=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
        s.record(); fn(); e.record(); e.synchronize(); ts.append(s.elapsed_time(e)/1e3)
    return statistics.median(ts)
for rows in (131072, 65536):
    H=1024
    x=torch.randn(rows,H,device='cuda').bfloat16()
    w=torch.randn(H,device='cuda'); b=torch.randn(H,device='cuda')
    for wg in (4,8,16,32):
        tune(0,wg)
        t=timeit(lambda: ops.layer_norm(x,w,b))
        print(json.dumps({"rows":rows,"fwd_wg_per_cu":wg,"us":round(t*1e6,1),"TBps":round(4*rows*H/t/1e12,2)}),flush=True)
    tune(0,8)
    xr=x.clone().requires_grad_(True); wr=w.clone().requires_grad_(True); br=b.clone().requires_grad_(True)
    y=ops.layer_norm(xr,wr,br); dy=torch.randn_like(y)
    for wg in (2,4,8):
        tune(1,wg)
        t=timeit(lambda: torch.autograd.grad(y,(xr,wr,br),dy,retain_graph=True))
        print(json.dumps({"rows":rows,"bwd_wg_per_cu":wg,"us":round(t*1e6,1),"TBps_6B":round(6*rows*H/t/1e12,2)}),flush=True)
    tune(1,4)
