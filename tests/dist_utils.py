"""Multi-process CPU (gloo) harness for the T1 test tier."""
import os
import socket
import traceback

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, errq, device="cpu", backend=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), MADNN_LOG_LEVEL="WARNING")
    torch.set_num_threads(1)
    import madnn

    try:
        madnn.init(device=device, backend=backend, timeout_s=120)
        fn(rank, world, *args)
    except Exception:  # noqa: BLE001
        errq.put((rank, traceback.format_exc()))
        raise
    finally:
        madnn.shutdown()


def run_dist(fn, world: int = 2, *args, device: str = "cpu", backend: str = None):
    """Run ``fn(rank, world, *args)`` in ``world`` gloo processes; re-raise the first failure.

    ``device="cuda"`` puts every rank on the (single) GPU of the box with a gloo group
    (RCCL refuses two ranks on one GPU), which exercises the device code paths."""
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, errq, device, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    if errs:
        raise AssertionError("rank %d failed:\n%s" % errs[0])
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    if bad:
        raise AssertionError(f"worker exit codes {bad}")
