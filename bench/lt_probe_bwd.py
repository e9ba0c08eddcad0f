"""hipBLASLt backward epilogues on gfx950 at GPT-2 medium's shapes (64 x 1024 tokens): DGELU /
DGELU_BGRAD (GELU backward fused into c_proj's data-grad GEMM, reading the saved pre-activation as
AUX) and BGRADA / BGRADB (a bias gradient out of a weight-gradient GEMM): how many algorithms the
heuristic offers.  python bench/lt_probe_bwd.py [--out file.json]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import madnn  # noqa: E402

EPI = {"DEFAULT": 1, "DGELU": 192, "DGELU_BGRAD": 208, "BGRADA": 256, "BGRADB": 512, "GELU_AUX_BIAS": 164}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    assert madnn.ops.load_kernels()
    ops = torch.ops.madnn
    dummy = torch.empty(65536 * 4096, device="cuda", dtype=torch.bfloat16)
    rows = []
    for (M, K, N) in [(65536, 1024, 4096), (65536, 4096, 1024), (4096, 65536, 1024), (3072, 65536, 1024)]:
        for name, e in EPI.items():
            for bc in (-1, 0, 2):
                for ac in (-1, 0, 2):
                    n = int(ops.lt_probe(M, N, K, e, bc, ac, False, dummy.data_ptr()))
                    rows.append({"M": M, "K": K, "N": N, "epi": name, "bias": bc, "aux": ac, "algos": n})
    ok = [r for r in rows if r["algos"] > 0 and r["epi"] != "DEFAULT"]
    print(json.dumps({"available": ok}, indent=None))
    if a.out:
        json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
