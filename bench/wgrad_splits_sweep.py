"""Split-count sweep of the K12W / K12W16 weight gradients (us per call) against madnn_wgrad_splits' choice;
one JSON line per shape (profiles/r6_wgrad_splits_sweep.jsonl)."""
import json, torch, sys, os
sys.path.insert(0, os.getcwd())
from madnn import ops
assert ops.load_kernels()
def timed(fn, reps=5):
    fn(); a=torch.cuda.Event(enable_timing=True); b=torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); a.record()
    for _ in range(reps): fn()
    b.record(); torch.cuda.synchronize(); return a.elapsed_time(b)/reps*1e3
for (M,N,K) in [(131072,50304,1024),(131072,4096,1024),(131072,1024,1024),(32768,50304,1024)]:
    dy=torch.randn(M,N,device="cuda").bfloat16(); x=torch.randn(M,K,device="cuda").bfloat16()
    out=torch.empty(N,K,device="cuda",dtype=torch.bfloat16)
    h=int(torch.ops.madnn.wgrad_splits(M,N,K))
    row={"shape":[M,N,K],"heuristic":h}
    for sp in sorted(set([1,2,3,4,5,6,8,10,12,16,h])):
        if M//64//sp < 8: continue
        row[f"w{sp}"]=round(timed(lambda: torch.ops.madnn.linear_wgrad4(dy,x,out,False,sp)),1)
        row[f"h{sp}"]=round(timed(lambda: torch.ops.madnn.linear_wgrad4h(dy,x,out,False,sp)),1)
    print(json.dumps(row), flush=True)
    del dy,x,out; torch.cuda.empty_cache()
