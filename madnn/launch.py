"""``python -m madnn.launch --nproc 8 script.py [args]`` — one process per GPU.

Replaces the reference's interactive ``mpirun -n N -npernode 1 --hostfile``
launcher (cifar_example/train.sh:1-16).  Single node, MI355X-first:

* spawns ``--nproc`` workers with RANK / LOCAL_RANK / WORLD_SIZE /
  MASTER_ADDR=127.0.0.1 / MASTER_PORT set (the same contract as
  ``torch.distributed.run``), plus ``HSA_ENABLE_IPC_MODE_LEGACY=0`` which the
  ROCm dmabuf IPC path for RCCL needs;
* optional CPU pinning of each worker to a contiguous core range;
* failure detection: if any worker exits non-zero (or is killed), all others
  are terminated and the launcher exits with that code — no half-dead job
  hanging in a collective;
* ``--fault rank:step:kind`` exports MADNN_FAULT for fault-injection tests
  (see ``madnn.utils.fault``).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m madnn.launch")
    ap.add_argument("--nproc", type=int, default=None, help="processes (default: visible GPUs or 1)")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--pin-cpus", action="store_true", help="pin each rank to a contiguous CPU range")
    ap.add_argument("--fault", default=None, help="rank:step:kind (raise|hang|exit) fault injection")
    ap.add_argument("--timeout", type=float, default=0.0, help="kill the job after this many seconds (0 = none)")
    ap.add_argument("-m", dest="module", action="store_true", help="run the target as a module")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    n = a.nproc
    if n is None:
        try:  # counting devices does not initialise HIP in this image
            import torch

            n = max(torch.cuda.device_count(), 1)
        except Exception:
            n = 1
    port = a.master_port or _free_port()
    base = dict(os.environ)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n), HSA_ENABLE_IPC_MODE_LEGACY="0")
    if a.fault:
        base["MADNN_FAULT"] = a.fault
    cmd = [sys.executable] + (["-m", a.script] if a.module else [a.script]) + a.args
    ncpu = os.cpu_count() or 1
    procs = []
    for r in range(n):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        pre = None
        if a.pin_cpus and hasattr(os, "sched_setaffinity"):
            per = max(ncpu // n, 1)
            cpus = set(range(r * per, min((r + 1) * per, ncpu))) or {r % ncpu}
            pre = (lambda c=cpus: os.sched_setaffinity(0, c))
        procs.append(subprocess.Popen(cmd, env=env, preexec_fn=pre, start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = [p for p in procs if p.poll() is None]
            failed = [p for p in procs if p.poll() not in (None, 0)]
            if failed:
                rc = failed[0].returncode or 1
                print(f"[madnn.launch] rank {procs.index(failed[0])} exited with {rc}; tearing down", file=sys.stderr)
                break
            if not alive:
                break
            if a.timeout and time.time() - t0 > a.timeout:
                print("[madnn.launch] timeout; tearing down", file=sys.stderr)
                rc = 124
                break
            time.sleep(0.2)
    except KeyboardInterrupt:
        rc = 130
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 10
        for p in procs:
            while p.poll() is None and time.time() < deadline:
                time.sleep(0.1)
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
    return rc


if __name__ == "__main__":
    sys.exit(main())
