"""In-process A/B of GPT-2 medium DP1 step variants (same box, same process, interleaved windows):

    python bench/gpt2_ab.py --batch 16 --windows 6 --steps 8 --switch lt_res

Variants toggle at run time (the model is built once):
  lt_res  : residual add in c_proj's hipBLASLt epilogue (on) vs a separate ATen add (off)
  gelu    : K11-family GELU forward kernel (on) vs ATen's F.gelu (off)
  wgrad   : weight gradients on the per-shape faster of hipBLASLt / K12 split-K (on) vs hipBLASLt (off)
  colsum  : attn-proj / c_proj bias grads from the next norm's backward column sums (on) vs their own pass (off)
  attn_colsum: qkv bias grad from the attention backward's dQKV column sums (on) vs its own pass (off)
  xent    : one-pass K6f cross entropy (loss + finished logit gradient in the forward) (on) vs two-pass K6 (off)
  gelu_fwd: c_fc forward on K12 with the fused bias + AUX + GELU epilogue (on) vs hipBLASLt + K11 GELU (off)
Prints a JSON line with the per-window ms/step and the median of each arm.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--windows", type=int, default=6)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--switch", default="lt_res",
                    choices=["lt_res", "gelu", "gelu_bwd_fast", "gelu_rcp", "native", "wgrad", "gelu_fwd", "colsum", "attn_colsum",
                             "xent"])
    ap.add_argument("--native", default="", help="FUNC:KEY:ON:OFF -- a native tunable, e.g. madnn_norm_tune:1:4:2")
    a = ap.parse_args()
    import madnn
    from madnn import ops
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.optim import FusedAdam

    madnn.init()
    torch.manual_seed(0)
    model = GPT2(gpt2_config("gpt2-medium"))
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
    eng, opt = madnn.distribute(model, opt, strategy="dp")
    ids = torch.randint(0, 50257, (a.batch, a.seq), device="cuda")

    def set_arm(on):
        if a.switch == "attn_colsum":
            ops.ATTN_COLSUM = on
        elif a.switch == "xent":
            ops.XENT_FUSED = on
        elif a.switch == "colsum":
            ops.NORM_COLSUM = on
        elif a.switch == "gelu_fwd":
            ops.GELU_FWD = "k12" if on else "lt"
        elif a.switch == "wgrad":  # per-shape timed hipBLASLt / K12 split-K (on) vs hipBLASLt only (off)
            ops.WGRAD = "auto" if on else "lt"
        elif a.switch == "lt_res":
            ops._LT_KIND["res"] = on
        elif a.switch == "gelu":
            ops.GELU_KERNEL = on
        elif a.switch == "gelu_bwd_fast":
            import ctypes

            ctypes.CDLL(str(ops.kernels_path())).madnn_bias_fast_tanh(1 if on else 0)
        elif a.switch == "native":
            import ctypes

            fn, key, von, voff = a.native.split(":")
            getattr(ctypes.CDLL(str(ops.kernels_path())), fn)(int(key), int(von if on else voff))
        elif a.switch == "gelu_rcp":
            import ctypes

            ctypes.CDLL(str(ops.kernels_path())).madnn_gelu_rcp(1 if on else 0)

    def window(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            eng.train_step(ids, ids)
            opt.step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    for arm in (True, False):
        set_arm(arm)
        window(3)
    res = {True: [], False: []}
    for w in range(a.windows):
        arm = (w % 2 == 0)
        set_arm(arm)
        res[arm].append(window(a.steps))
    out = {"switch": a.switch, "native": a.native, "batch": a.batch, "on_ms": res[True], "off_ms": res[False],
           "on_median": statistics.median(res[True]), "off_median": statistics.median(res[False]),
           "lt_failed": {str(k): str(v)[:100] for k, v in ops._LT_FAILED.items()}}
    out["gain_pct"] = 100.0 * (out["off_median"] - out["on_median"]) / out["off_median"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
