"""Which hipBLASLt epilogues exist on gfx950 for GPT-2 medium's MLP shapes, and what they cost
vs the unfused GEMM + elementwise passes.  python bench/lt_probe.py [--out file.json]"""
import argparse
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import madnn  # noqa: E402

EPI = {"DEFAULT": 1, "BIAS": 4, "GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160, "GELU_AUX_BIAS": 164}


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    assert madnn.ops.load_kernels()
    ops = torch.ops.madnn
    res = {"probe": [], "timing_us": {}}
    dummy = torch.empty(16384 * 4096, device="cuda", dtype=torch.bfloat16)
    for (M, K, N) in [(16384, 1024, 4096), (16384, 4096, 1024)]:
        for name, e in EPI.items():
            for bc in (-1, 0, 2):
                for ac in (-1, 0, 2):
                    for ptr in (0, dummy.data_ptr()):
                        n = int(ops.lt_probe(M, N, K, e, bc, ac, False, ptr))
                        res["probe"].append({"M": M, "K": K, "N": N, "epi": name, "bias": bc, "aux": ac,
                                             "ptr": bool(ptr), "algos": n})
    M, K, N = 16384, 1024, 4096
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.03
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    r = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    t = res["timing_us"]
    t["F.linear(bias)"] = timeit(lambda: F.linear(x, w, b))
    t["F.linear+gelu"] = timeit(lambda: F.gelu(F.linear(x, w, b), approximate="tanh"))
    t["F.linear+add"] = timeit(lambda: F.linear(x, w, b) + r)
    for nm, kw in {"lt bias": dict(residual=None, gelu=False), "lt bias+residual": dict(residual=r, gelu=False),
                   "lt gelu_aux_bias": dict(residual=None, gelu=True)}.items():
        try:
            t[nm] = timeit(lambda: ops.lt_linear(x, w, b, kw["residual"], kw["gelu"], kw["gelu"]))
        except RuntimeError as e:
            t[nm] = str(e)[:160]
    ok = [p for p in res["probe"] if p["algos"] > 0 and "AUX" in p["epi"]]
    print(json.dumps({"gelu_supported": ok[:12], "timing_us": t}, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
