"""Weight-gradient GEMM A/B: K12 (8 waves, ``linear_wgrad``) vs K12W (4 waves, one per SIMD,
``linear_wgrad4``) vs hipBLASLt (torch.matmul), same operands, interleaved timing; K12W checked
against an fp32 reference first.

    python bench/gemm_wgrad_ab.py --out gpurun_out/wgrad_ab.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, tokens M, out features N, in features K)
SHAPES = [
    ("gpt2m c_fc", 131072, 4096, 1024), ("gpt2m c_proj", 131072, 1024, 4096),
    ("gpt2m qkv", 131072, 3072, 1024), ("gpt2m attn_proj", 131072, 1024, 1024),
    ("gpt2m lm_head", 131072, 50304, 1024),
    ("gpt2m c_fc mb32", 32768, 4096, 1024), ("gpt2m lm_head mb32", 32768, 50304, 1024),
    ("bert-l fc1", 65536, 4096, 1024), ("bert-l out", 65536, 1024, 4096),
    ("llama8b gate_up", 16384, 28672, 4096), ("llama8b down", 16384, 4096, 14336),
    ("llama8b qkv", 16384, 6144, 4096), ("llama8b o", 16384, 4096, 4096),
    ("square 8192", 8192, 8192, 8192),
    # ResNet-50 1x1 convolution weight gradients at 2048 images (rows = pixels, N = cout, K = cin)
    ("r50 conv 56 64->256", 6422528, 256, 64), ("r50 conv 56 256->64", 6422528, 64, 256),
    ("r50 conv 28 512->128", 1605632, 128, 512), ("r50 conv 28 128->512", 1605632, 512, 128),
    ("r50 conv 14 1024->256", 401408, 256, 1024), ("r50 conv 14 256->1024", 401408, 1024, 256),
    ("r50 conv 7 2048->512", 100352, 512, 2048), ("r50 conv 7 512->2048", 100352, 2048, 512),
]


def timed(fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    from madnn import ops

    assert ops.load_kernels()
    w12 = torch.ops.madnn.linear_wgrad
    w12w = torch.ops.madnn.linear_wgrad4
    torch.manual_seed(0)
    rows = []
    try:
        # correctness of K12W first (fp32 reference on a few thousand tokens; ragged N / K tiles)
        for M, N, K in [(4096, 1024, 512), (2048, 4104, 1000), (8192, 768, 3072), (64 * 33, 520, 264)]:
            dy = (torch.randn(M, N, device="cuda") * 0.5).bfloat16()
            x = torch.randn(M, K, device="cuda").bfloat16()
            ref = dy.float().t() @ x.float()
            for sp in (1, 3):
                w = w12w(dy, x, None, False, sp)
                acc = w12w(dy, x, w.clone(), True, sp)
                rel = float((w.float() - ref).norm() / ref.norm())
                rel_acc = float((acc.float() - 2 * ref).norm() / (2 * ref).norm())
                print(f"check M={M} N={N} K={K} splits={sp}: rel {rel:.2e} accumulate rel {rel_acc:.2e}", flush=True)
                assert rel < 1e-2 and rel_acc < 1e-2, (M, N, K, sp, rel, rel_acc)
        for name, M, N, K in SHAPES:
            if args.only and args.only not in name:
                continue
            dy = torch.randn(M, N, device="cuda").bfloat16()
            x = torch.randn(M, K, device="cuda").bfloat16()
            flop = 2.0 * M * N * K
            sp = int(torch.ops.madnn.wgrad_splits(M, N, K))
            out = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)

            t = {}
            w0 = w12(dy, x, None, False, 0)
            w1 = w12w(dy, x, None, False, 0)
            diff = float((w0.float() - w1.float()).norm() / w0.float().norm())
            if M % 128 == 0:   # K12W16 against K12
                w2 = torch.ops.madnn.linear_wgrad4h(dy, x, None, False, 0)
                diff16 = float((w0.float() - w2.float()).norm() / w0.float().norm())
                assert diff16 < 1e-2, (name, diff16)
            for rnd in range(2):          # interleaved: K12, K12W, K12W16, hipBLASLt, twice
                t.setdefault("k12", []).append(timed(lambda: w12(dy, x, out, False, 0), args.reps))
                t.setdefault("k12w", []).append(timed(lambda: w12w(dy, x, out, False, 0), args.reps))
                if M % 128 == 0:
                    t.setdefault("k12wh", []).append(
                        timed(lambda: torch.ops.madnn.linear_wgrad4h(dy, x, out, False, 0), args.reps))
                t.setdefault("lt", []).append(timed(lambda: torch.mm(dy.t(), x, out=out), args.reps))
            best = {k: min(v) for k, v in t.items()}
            row = {"shape": name, "M": M, "N": N, "K": K, "splits": sp, "k12w_vs_k12_rel": float(f"{diff:.3g}")}
            for k, us in best.items():
                row[k + "_us"] = round(us, 1)
                row[k + "_tflops"] = round(flop / us / 1e6, 1)
            row["k12w_speedup"] = round(best["k12"] / best["k12w"], 3)
            rows.append(row)
            print(json.dumps(row), flush=True)
            del dy, x, out, w0, w1
            torch.cuda.empty_cache()
    finally:
        pass
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
