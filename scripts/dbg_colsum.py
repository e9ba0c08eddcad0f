import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, madnn
from madnn import ops
torch.manual_seed(0)
B, S, E, H, D = 2, 256, 256, 4, 64
x = torch.randn(B, S, E, device="cuda", dtype=torch.bfloat16, requires_grad=True)
w = (torch.randn(3 * H * D, E, device="cuda") * 0.06).bfloat16().requires_grad_()
b = torch.zeros(3 * H * D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
y = ops.linear(x, w, b)
print("y.grad_fn", type(y.grad_fn).__name__, getattr(y.grad_fn, "bias_dtype", "NA"))
qkv = y.view(B, S, 3 * H, D)
print("qkv._base is y", qkv._base is y, "from_biased(base)", ops._from_biased_linear(qkv._base))
o = ops.attention_qkvpacked(qkv, H, H, causal=True)
print("o.grad_fn", type(o.grad_fn).__name__, "ctx.colsum", getattr(o.grad_fn, "colsum", "NA"))
orig = ops._AttnPackedFn.backward
def bw(ctx, do):
    r = orig(ctx, do)
    print("attn bwd: colsum attr", hasattr(r[0], "_madnn_colsum"))
    return r
ops._AttnPackedFn.backward = staticmethod(bw)
origl = ops._LinearFn.backward
def lbw(ctx, g):
    print("lin bwd: g attr", hasattr(g, "_madnn_colsum"), "base", g._base is not None, hasattr(g._base, "_madnn_colsum") if g._base is not None else None)
    return origl(ctx, g)
ops._LinearFn.backward = staticmethod(lbw)
o.float().sum().backward()
