"""MI355X machine model used by the cost model.

Defaults are the measured / guide numbers for one MI355X (gfx950) and its
xGMI mesh (MI355X_MICROARCH.md: 6.3 TB/s achievable HBM3E, ~2.5 PF dense
bf16 MFMA; task spec: 7 xGMI links x ~153 GB/s per GPU).  ``load()`` overlays
a JSON file written by ``madnn.comm.bench`` / ``madnn.planner.calibrate``
(env ``MADNN_HW_PROFILE``) so the planner prices collectives with numbers
measured on the actual node rather than datasheet values.
"""
from __future__ import annotations

import json
import os
from dataclasses import asdict, dataclass


@dataclass
class Machine:
    name: str = "MI355X"
    hbm_gb: float = 288.0
    hbm_tbps: float = 5.5            # achievable streaming (6.29 measured float4 copy; ~88% typical for kernels)
    bf16_tflops: float = 1100.0      # sustained GEMM-heavy training (~45% of 2.5 PF dense peak)
    fp32_tflops: float = 120.0
    link_gbps: float = 153.0         # one xGMI link, one direction
    links: int = 7
    allreduce_eff: float = 0.75      # fraction of the ring bound RCCL reaches on large buckets
    p2p_gbps: float = 60.0           # achievable point-to-point over one link (send/recv)
    collective_latency_us: float = 25.0
    kernel_launch_us: float = 4.0

    def allreduce_s(self, nbytes: float, world: int) -> float:
        """Ring all-reduce time: 2(W-1)/W * bytes over the per-GPU xGMI bandwidth RCCL spreads on.

        RCCL runs several channels over distinct links; on a fully connected
        8-GPU mesh the usable per-GPU bandwidth for one collective approaches
        (W-1) links, capped at the link count."""
        if world <= 1:
            return 0.0
        bw = self.link_gbps * 1e9 * min(self.links, world - 1) * self.allreduce_eff
        return 2.0 * (world - 1) / world * nbytes / bw + self.collective_latency_us * 1e-6

    def p2p_s(self, nbytes: float) -> float:
        return nbytes / (self.p2p_gbps * 1e9) + self.collective_latency_us * 1e-6


_CACHE = {}


def load() -> Machine:
    path = os.environ.get("MADNN_HW_PROFILE")
    key = path or ""
    if key in _CACHE:
        return _CACHE[key]
    m = Machine()
    if path and os.path.exists(path):
        with open(path) as f:
            for k, v in json.load(f).items():
                if hasattr(m, k):
                    setattr(m, k, type(getattr(m, k))(v))
    _CACHE[key] = m
    return m


def dump(m: Machine, path: str) -> None:
    with open(path, "w") as f:
        json.dump(asdict(m), f, indent=2)
