#!/usr/bin/env python3
"""A/B: ResNet-50's stride-1 1x1 convolutions (NHWC bf16) on MIOpen vs hipBLASLt GEMMs vs madnn K9.

A stride-1 1x1 conv over an NHWC tensor is exactly x[M, Cin] @ W[Cout, Cin]^T with
M = N*H*W; forward, data-grad and weight-grad are three GEMMs.  Times each pass per
shape (min over interleaved rounds of median event timings, one process —
cdna_hip_programming.md §5.4 rule 24), checks K9 against the fp32 result, and prints
one JSON line per shape plus per-step totals (each shape weighted by how often a
ResNet-50 step runs it).

    python bench/conv1x1_vs_gemm.py [N=512] [--json out.json]
"""
import json
import statistics
import sys

import torch
import torch.nn.functional as F


def t_of(fn, iters=10):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


# (H=W, Cin, Cout, count per ResNet-50 step)
SHAPES = [(56, 64, 64, 1), (56, 64, 256, 4), (56, 256, 64, 2), (56, 256, 128, 1), (28, 128, 512, 4),
          (28, 512, 128, 3), (28, 512, 256, 1), (14, 256, 1024, 6), (14, 1024, 256, 5), (14, 1024, 512, 1),
          (7, 512, 2048, 3), (7, 2048, 512, 2)]


def main():
    import madnn

    madnn.init()
    assert madnn.ops.load_kernels()
    args = [a for a in sys.argv[1:] if not a.startswith("--") and not a.endswith(".json")]
    N = int(args[0]) if args else 512
    out = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    dev = "cuda"
    rows = []
    passes = ("fwd", "dgrad", "wgrad")
    tot = {k: {p: 0.0 for p in passes} for k in ("miopen", "gemm", "k9")}
    for hw, cin, cout, cnt in SHAPES:
        torch.manual_seed(0)
        x = torch.randn(N, cin, hw, hw, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device=dev) * cin ** -0.5).bfloat16().contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(N, cout, hw, hw, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        w2 = w.reshape(cout, cin)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        cb = torch.ops.aten.convolution_backward
        fns = {
            ("miopen", "fwd"): lambda: F.conv2d(x, w),
            ("miopen", "dgrad"): lambda: cb(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1,
                                            (True, False, False)),
            ("miopen", "wgrad"): lambda: cb(dy, x, w, None, (1, 1), (0, 0), (1, 1), False, (0, 0), 1,
                                            (False, True, False)),
            ("gemm", "fwd"): lambda: torch.mm(x2, w2.t()),
            ("gemm", "dgrad"): lambda: torch.mm(dy2, w2),
            ("gemm", "wgrad"): lambda: torch.mm(dy2.t(), x2),
            ("k9", "fwd"): lambda: torch.ops.madnn.conv1x1_fwd(x, w, True),
            ("k9", "dgrad"): lambda: torch.ops.madnn.conv1x1_dgrad(dy, w),
            ("k9", "wgrad"): lambda: torch.ops.madnn.conv1x1_wgrad(dy, x),
        }
        # numerics of K9 against fp32 GEMMs on this shape
        err = {}
        y, _ = torch.ops.madnn.conv1x1_fwd(x, w, False)
        ref = x2.float() @ w2.float().t()
        err["fwd"] = ((y.permute(0, 2, 3, 1).reshape(-1, cout).float() - ref).abs().max() / ref.abs().max()).item()
        ref = dy2.float() @ w2.float()
        dx = torch.ops.madnn.conv1x1_dgrad(dy, w)
        err["dgrad"] = ((dx.permute(0, 2, 3, 1).reshape(-1, cin).float() - ref).abs().max() / ref.abs().max()).item()
        ref = dy2.float().t() @ x2.float()
        err["wgrad"] = ((torch.ops.madnn.conv1x1_wgrad(dy, x) - ref).abs().max() / ref.abs().max()).item()
        del ref, y, dx
        best = {k: [] for k in fns}
        for _ in range(3):
            for k, f in fns.items():
                best[k].append(t_of(f))
        r = {f"{k[0]}_{k[1]}": round(min(v), 4) for k, v in best.items()}
        r.update(shape=[hw, cin, cout], count=cnt, M=N * hw * hw, k9_max_rel_err=err)
        for k in tot:
            for p in passes:
                tot[k][p] += cnt * r[f"{k}_{p}"]
        rows.append(r)
        print(json.dumps(r), flush=True)
    summary = {"N": N, "per_step_ms": {k: {p: round(v, 3) for p, v in d.items()} | {"total": round(sum(d.values()), 3)}
                                       for k, d in tot.items()}}
    print(json.dumps(summary), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump({"rows": rows, **summary}, f, indent=1)


if __name__ == "__main__":
    main()
