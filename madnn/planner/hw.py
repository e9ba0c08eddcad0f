"""MI355X machine model used by the cost model.

Defaults are the guide numbers for one MI355X (gfx950) and its xGMI mesh
(MI355X_MICROARCH.md: 6.3 TB/s achievable HBM3E, ~2.5 PF dense bf16 MFMA; task
spec: 7 xGMI links x ~153 GB/s per GPU).  ``load()`` overlays, in order of
precedence, the JSON profile named by ``MADNN_HW_PROFILE``, the node's own
profile written by ``madnn.planner.calibrate`` (``~/.cache/madnn/hw_profile.json``),
or the profile shipped in-tree (``madnn/tuning/hw_mi355x.json``, measured on an
MI355X box with ``calibrate``), so the planner prices compute and collectives
with measured numbers rather than datasheet values.
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
    calibrated: str = ""             # when / at what world size the profile was measured ("" = datasheet)
    source: str = "defaults"

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


def host_cpu() -> Machine:
    """A rough host-CPU profile for jobs that really run on CPU over gloo (tests, the MLP
    config): pricing their compute with MI355X numbers would make every collective look
    expensive and push the planner to tensor parallelism for convolutional nets."""
    return Machine(name="host-cpu", hbm_gb=64.0, hbm_tbps=0.02, bf16_tflops=0.2, fp32_tflops=0.2, link_gbps=1.0,
                   links=1, allreduce_eff=1.0, p2p_gbps=1.0, collective_latency_us=300.0, kernel_launch_us=20.0,
                   source="host-cpu")


_CACHE = {}
SHIPPED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "hw_mi355x.json")


def default_profile_path() -> str:
    return os.path.join(os.path.expanduser("~"), ".cache", "madnn", "hw_profile.json")


def profile_candidates():
    return [p for p in (os.environ.get("MADNN_HW_PROFILE"), default_profile_path(), SHIPPED) if p]


def invalidate() -> None:
    _CACHE.clear()


def load() -> Machine:
    """The machine model: the first existing profile of :func:`profile_candidates` over the
    defaults.  A single-GPU profile leaves the link numbers at their defaults; one measured
    with several ranks overrides them too."""
    paths = profile_candidates()
    key = tuple(paths)
    if key in _CACHE:
        return _CACHE[key]
    m = Machine()
    for path in paths:
        if os.path.exists(path):
            with open(path) as f:
                for k, v in json.load(f).items():
                    if hasattr(m, k) and k != "source":
                        setattr(m, k, type(getattr(m, k))(v))
            m.source = path
            break
    _CACHE[key] = m
    return m


def dump(m: Machine, path: str) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(asdict(m), f, indent=2)
