#!/usr/bin/env python3
"""A/B the K11 fused Linear backward (bias gradient + tanh-GELU backward in one pass) against
ATen's (GELU backward + column-sum reduce) inside the GPT-2 medium DP1 training step,
batch 16 x 1024, one process, configurations interleaved round-robin."""
import json
import statistics
import time

import torch


def main():
    import madnn
    from madnn import ops
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.optim import FusedAdam

    madnn.init()
    import ctypes

    tune = ctypes.CDLL(str(ops.kernels_path())).madnn_bias_tune
    kern = {}
    for n in (1024, 3072, 4096):
        dy = torch.randn(16384, n, device="cuda").bfloat16()
        pre = torch.randn(16384, n, device="cuda").bfloat16()

        def t(fn, it=20):
            fn()
            s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s_.record()
            for _ in range(it):
                fn()
            e_.record()
            e_.synchronize()
            return round(s_.elapsed_time(e_) / it * 1e3, 1)

        for wg in (1, 2, 4, 8):
            old = (tune(0, wg), tune(1, wg))
            kern[f"{n}_wg{wg}"] = {"k11_sum_us": t(lambda: ops.bias_grad(dy, None, torch.bfloat16)),
                                   "k11_gelu_us": t(lambda: ops.bias_grad(dy, pre, torch.bfloat16))}
            tune(0, old[0])
            tune(1, old[1])
        kern[n] = {"k11_sum_us": t(lambda: ops.bias_grad(dy, None, torch.bfloat16)),
                   "aten_sum_us": t(lambda: dy.sum(0)),
                   "k11_gelu_us": t(lambda: ops.bias_grad(dy, pre, torch.bfloat16)),
                   "aten_gelu_us": t(lambda: torch.ops.aten.gelu_backward(dy, pre, approximate="tanh").sum(0))}
    print(json.dumps(kern), flush=True)
    torch.manual_seed(0)
    cfg = gpt2_config("gpt2-medium")
    model = GPT2(cfg)
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
    eng, opt = madnn.distribute(model, opt, strategy="dp")
    ids, _ = madnn.data.synthetic_batch("tokens", 16, madnn.device(), seq_len=1024, vocab=cfg.vocab_size)

    def step():
        loss = eng.train_step(ids, ids)
        opt.step()
        return loss

    for _ in range(4):
        step()
    times = {True: [], False: []}
    for rnd in range(5):
        for on in (False, True):
            ops.FUSED_LINEAR = on
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(4):
                loss = step()
            torch.cuda.synchronize()
            times[on].append((time.perf_counter() - t0) / 4 * 1e3)
        print(json.dumps({"aten": round(times[False][-1], 3), "k11": round(times[True][-1], 3),
                          "loss": float(loss)}), flush=True)
    res = {("k11" if k else "aten"): {"median_ms": round(statistics.median(v), 3), "min_ms": round(min(v), 3),
                                      "tok_s": round(16 * 1024 / statistics.median(v) * 1e3)}
           for k, v in times.items()}
    res["kernels"] = kern
    print(json.dumps(res), flush=True)
    with open("gpurun_out/linear_ab.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
