"""Linear data gradient dX = dY W on the GPT-2 / BERT / Llama shapes: PyTorch's matmul (hipBLASLt),
madnn's own hipBLASLt plan (``lt_linear(..., w_kn=True)``) and K12WD (``linear_dgrad4``: the K12W
engine with dY as a row image), same operands, interleaved rounds.  One JSON line per shape (us)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # name, tokens M, reduction N (out features), K (in features)
    ("gpt2m qkv", 131072, 3072, 1024), ("gpt2m attn_proj", 131072, 1024, 1024), ("gpt2m c_fc", 131072, 4096, 1024),
    ("gpt2m c_proj", 131072, 1024, 4096), ("gpt2m lm_head", 131072, 50304, 1024), ("gpt2m qkv mb32", 32768, 3072, 1024),
    ("gpt2m c_fc mb32", 32768, 4096, 1024), ("bert-l fc1", 65536, 4096, 1024), ("llama8b down", 16384, 4096, 14336),
    ("llama8b gate_up", 16384, 28672, 4096), ("llama8b o", 16384, 4096, 4096),
]


def timed(fn, reps=10):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    from madnn import ops

    assert ops.load_kernels()
    rows = []
    for name, M, N, K in SHAPES:
        dy = torch.randn(M, N, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.03).bfloat16()
        ref = dy.float() @ w.float() if M * K * 4 < 4e9 else None
        d = torch.ops.madnn.linear_dgrad4(dy, w)
        if ref is not None:
            rel = float((d.float() - ref).norm() / ref.norm())
            assert rel < 1e-2, (name, rel)
            del ref
        cands = {"lt": lambda: dy @ w,
                 "ltk": lambda: torch.ops.madnn.lt_linear(dy, w, None, None, False, False, True)[0],
                 "k12wd": lambda: torch.ops.madnn.linear_dgrad4(dy, w)}
        t = {}
        for _ in range(2):
            for k, f in cands.items():
                t.setdefault(k, []).append(timed(f))
        row = {"shape": name, "M": M, "N": N, "K": K}
        for k, v in t.items():
            row[k + "_us"] = round(min(v), 1)
            row[k + "_tflops"] = round(2.0 * M * N * K / min(v) / 1e6, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del dy, w, d
        torch.cuda.empty_cache()
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
