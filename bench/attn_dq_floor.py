"""Is a one-pass attention backward (dQ accumulated with f32 atomics inside the dK / dV kernel)
worth building on MI355X?  Times, at the bench shapes, (1) the atomic traffic alone that such a
kernel must issue (``madnn_dq_atomic_floor``, probe.hip: one global_atomic_add_f32 per dQ element
per key block, nothing else) and (2) the whole current two-kernel backward, plus the separate dQ
kernel's share of it from the steady-step table.  If (1) exceeds the dQ kernel it would replace,
the fused design loses whatever its MFMA savings.

    python bench/attn_dq_floor.py --out gpurun_out/attn_dq_floor.json
"""
import argparse
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    from madnn import ops

    assert ops.load_kernels()
    lib = ctypes.CDLL(str(ops.kernels_path()))
    fn = lib.madnn_dq_atomic_floor
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_void_p]
    fn.restype = ctypes.c_int
    rows = []
    # (name, B, S, H, Hkv, D): GPT-2 medium b128 (the bench), Llama-3 8B (4 x 4096, GQA 32 / 8)
    for name, B, S, H, HKV, D in [("gpt2m_b128", 128, 1024, 16, 16, 64), ("llama3_8b", 4, 4096, 32, 8, 128)]:
        dq = torch.zeros(B * H, S, D, device="cuda", dtype=torch.float32)
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        floor = {}
        for kblock in (128, 256):
            floor[kblock] = timed(lambda: fn(dq.data_ptr(), B * H, S, D, kblock, 1, stream))
        adds = {kb: sum(S - j * kb for j in range((S + kb - 1) // kb)) * D * B * H for kb in (128, 256)}
        q = torch.randn(B, S, H, D, device="cuda").bfloat16().requires_grad_(True)
        k = torch.randn(B, S, HKV, D, device="cuda").bfloat16().requires_grad_(True)
        v = torch.randn(B, S, HKV, D, device="cuda").bfloat16().requires_grad_(True)
        o = ops.attention(q, k, v, causal=True)
        do = torch.randn_like(o)
        fwd = timed(lambda: ops.attention(q, k, v, causal=True))
        bwd_total = timed(lambda: torch.autograd.grad(ops.attention(q, k, v, causal=True), (q, k, v), do)) - fwd
        rows.append({"shape": name, "B": B, "S": S, "H": H, "Hkv": HKV, "D": D,
                     "atomic_floor_us": {str(kb): round(t, 1) for kb, t in floor.items()},
                     "atomic_bytes_GB": {str(kb): round(n * 4 / 1e9, 3) for kb, n in adds.items()},
                     "atomic_TBps": {str(kb): round(adds[kb] * 4 / (floor[kb] * 1e-6) / 1e12, 2) for kb in floor},
                     "fwd_us": round(fwd, 1), "bwd_two_kernel_us": round(bwd_total, 1)})
        print(json.dumps(rows[-1]), flush=True)
        del dq, q, k, v, o, do
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
