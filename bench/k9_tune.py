#!/usr/bin/env python3
"""Sweep K9's launch tunables (XCD remap, persistent grid size, weight-grad split count) on
ResNet-50's 1x1 shapes at batch 512; one process, interleaved (cdna_hip_programming.md §5.4 rule 24)."""
import ctypes
import json
import statistics
import sys

import torch


def t_of(fn, iters=8):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return statistics.median(ts)


SHAPES = [(56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024), (14, 1024, 256),
          (7, 512, 2048), (7, 2048, 512)]


def main():
    import madnn

    madnn.init()
    assert madnn.ops.load_kernels()
    lib = ctypes.CDLL(str(madnn.ops.kernels_path()))
    tune = lib.madnn_conv1x1_tune
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    fwd_cfg = [(x, wg) for x in (0, 1) for wg in (256, 512, 1024, 4096)]
    wg_cfg = [(x, wg) for x in (0, 1) for wg in (256, 512, 1024)]
    out = []
    for hw, cin, cout in SHAPES:
        x = torch.randn(N, cin, hw, hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device="cuda") * cin ** -0.5).bfloat16()
        dy = torch.randn(N, cout, hw, hw, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        r = {"shape": [hw, cin, cout]}
        for xc, wg in fwd_cfg:
            tune(2, xc)
            tune(0, wg)
            r[f"fwd_x{xc}_g{wg}"] = round(min(t_of(lambda: torch.ops.madnn.conv1x1_fwd(x, w, True)) for _ in range(2)), 4)
            r[f"dgrad_x{xc}_g{wg}"] = round(min(t_of(lambda: torch.ops.madnn.conv1x1_dgrad(dy, w)) for _ in range(2)), 4)
        tune(0, 512)
        for xc, wg in wg_cfg:
            tune(2, xc)
            tune(1, wg)
            r[f"wgrad_x{xc}_g{wg}"] = round(min(t_of(lambda: torch.ops.madnn.conv1x1_wgrad(dy, x)) for _ in range(2)), 4)
        tune(1, 256)
        tune(2, 1)
        out.append(r)
        print(json.dumps(r), flush=True)
    with open("gpurun_out/k9_tune.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
