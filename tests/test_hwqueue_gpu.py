"""The hardware-queue probe kernels (madnn/ops/csrc/probe.hip) on the device.

The probe is what showed that HIP streams of one process share GPU_MAX_HW_QUEUES hardware
queues and serialise across them (profiles/r4_hwqueue_probe_q4.json), the reason the pipeline
transport is built to complete even fully serialised (madnn/parallel/pp.py: issue_plan).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pair(wait_stream, set_stream, value, timeout_us):
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = torch.zeros(2, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(wait_stream):
        torch.ops.madnn.hwq_wait(flag, value, timeout_us, out)
    with torch.cuda.stream(set_stream):
        torch.ops.madnn.hwq_set(flag, value)
    torch.cuda.synchronize()
    return out.tolist()


def test_probe_wait_is_bounded_behind_its_own_setter(cuda):
    """Waiter and setter on ONE stream: the setter runs only after the waiter gave up, so the
    waiter reports a timeout after ~timeout_us -- the bounded spin cannot hang the queue."""
    import madnn.ops as ops

    assert ops.load_kernels()
    s = torch.cuda.Stream()
    ok, ticks = _pair(s, s, 7, 2000)
    assert ok == 0 and 150_000 <= ticks <= 2_000_000   # 100 MHz ticks: >= 1.5 ms waited


def test_probe_sees_a_setter_on_another_priority_queue(cuda):
    """The high-priority stream pool has hardware queues of its own (measured: default and
    low-priority streams never share one with it), so a setter there reaches a waiter on the
    compute stream within microseconds."""
    import madnn.ops as ops

    assert ops.load_kernels()
    ok, ticks = _pair(torch.cuda.default_stream(), torch.cuda.Stream(priority=-1), 11, 200_000)
    assert ok == 1 and ticks < 10_000_000


@pytest.mark.parametrize("lag", [0.0, 0.3])
@pytest.mark.parametrize("kind,V", [("gpipe", 1), ("1f1b", 1), ("interleaved", 2)])
def test_engine_pipeline_program_completes_on_real_hw_queues(cuda, kind, V, lag):
    """Both ranks of an S = 2 pipeline replayed on this GPU's hardware queues (one queue pool
    per rank, seven streams each, rendezvous messages): both of madnn's issue plans complete
    without a timed-out message."""
    import madnn.ops as ops
    from madnn.utils.hwqueue import replay

    assert ops.load_kernels()
    rec = replay(kind, V, 8, "engine", spin_us=100, timeout_us=200000,
                 epoch=100 + V + (kind == "gpipe") + (10 if lag else 0), lag=lag)
    assert rec["timed_out"] == 0 and rec["unset"] == 0, rec


_CHILD = r"""
import json, sys
sys.path.insert(0, {root!r})
import torch
import madnn.ops as ops
from madnn.utils.hwqueue import replay
assert ops.load_kernels()
out = []
for design, lag in (("engine", 0.0), ("engine", 0.3), ("prepost", 0.0)):
    out.append(replay("1f1b", 1, 8, design, spin_us=100, timeout_us=100000, epoch=1 + len(out), lag=lag))
print("RESULT " + json.dumps(out), flush=True)
"""


@pytest.mark.parametrize("queues", [1, 2])
def test_replay_negative_control_at_few_hw_queues(queues):
    """The replay can fail for the reason it guards against: with GPU_MAX_HW_QUEUES = 1 (set
    before the child process touches the GPU) every stream of a replayed rank shares one hardware
    queue -- the fully serialised setting of the transport's safety argument (pp.issue_plan) --
    and the round-3 design that posts every receive up front deadlocks (its messages time out),
    while both of the engine's issue plans complete.  At 2 queues the engine plans complete too."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(queues))
    res = subprocess.run([sys.executable, "-c", _CHILD.format(root=root)], env=env, capture_output=True, text=True,
                         timeout=100)
    assert res.returncode == 0, res.stderr[-3000:]
    line = [ln for ln in res.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    eng0, eng_lag, prepost = json.loads(line[len("RESULT "):])
    for rec in (eng0, eng_lag):
        assert rec["timed_out"] == 0 and rec["unset"] == 0, rec
    if queues == 1:
        assert prepost["timed_out"] > 0, prepost
