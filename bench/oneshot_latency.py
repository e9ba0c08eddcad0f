"""K5 one-shot all-reduce latency: W processes on the box's GPU(s) (gloo group for the IPC handle
exchange only), per-call time of the one kernel for message sizes 4 KB .. 4 MB, bf16.

    python bench/oneshot_latency.py --world 2 --iters 200 --json-out gpurun_out/oneshot_latency.json

On a one-GPU box the W ranks share the device, so the staged reads hit local HBM instead of
xGMI; the number is the protocol's floor (launch + flag round trip + W-way sum), not a link
measurement."""
import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, iters, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(rank % torch.cuda.device_count())
    from madnn.comm.oneshot import OneShotAllReduce

    c = OneShotAllReduce(None, cap_bytes=8 << 20)
    out = {}
    for kb in (4, 16, 64, 256, 1024, 4096):
        x = torch.randn(kb * 512, device="cuda").bfloat16()
        for _ in range(10):
            c(x)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            c(x)
        torch.cuda.synchronize()
        out[kb] = (time.perf_counter() - t0) / iters * 1e6
    c.check()
    dist.barrier()
    c.close()
    q.put((rank, out))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, a.world, port, a.iters, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(a.world))
    for p in ps:
        p.join(60)
    line = json.dumps({"world": a.world, "devices": torch.cuda.device_count(), "dtype": "bf16",
                       "us_per_call_by_kb": {k: max(res[r][k] for r in res) for k in res[0]}})
    print(line)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
