"""The driver's bench.py contract on the device with 2 ranks (torch.distributed.run).

The box has one GPU and RCCL refuses two ranks per GPU, so both ranks share it over a gloo
group (``--backend gloo``); everything else is the multi-GPU path the driver's scaling run takes:
DP with overlapped bucket reductions (ResNet-50) and the 2-stage GPT-2 medium pipeline, timed
between barriers, max over ranks, one JSON line from rank 0."""
import json
import os
import subprocess
import sys

import pytest

from dist_utils import free_port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--backend", "gloo"] + extra
    env = dict(os.environ, MADNN_LOG_LEVEL="WARNING", OMP_NUM_THREADS="4")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["dtype"] == "bf16" and res["value"] > 0
    return res


def test_bench_resnet50_dp2_on_device(cuda):
    res = _run(["--model", "resnet50", "--batch", "16", "--image-size", "64"])
    assert res["config"]["parallelism"] == "dp2" and res["config"]["global_batch"] == 32
    assert res["scaling"] == "weak"


def test_bench_gpt2_medium_pp2_on_device(cuda):
    res = _run(["--model", "gpt2-medium", "--gpt2-batch-per-gpu", "2", "--seq-len", "128", "--microbatches", "2"])
    assert res["config"]["parallelism"] == "pp2" and res["scaling"] == "weak"
    assert res["gpt2_pp"]["microbatches"] == 2


def _run_rccl_world1(cmd_head, extra):
    cmd = cmd_head + ["bench.py", "--gpus", "1", "--steps", "2", "--warmup", "1", "--batch", "32",
                      "--image-size", "64", "--gpt2-batch-per-gpu", "2", "--seq-len", "128"] + extra
    env = dict(os.environ, MADNN_LOG_LEVEL="WARNING", OMP_NUM_THREADS="4")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    # the whole metric in one line, both halves on the real RCCL communicator
    assert res["config"]["process_group"] == "nccl", res["config"]
    assert res["config"]["parallelism"] == "dp1" and res["value"] > 0
    assert res["gpt2_pp"]["parallelism"] == "dp1" and res["gpt2_pp"]["tokens_per_s"] > 0
    return res


def test_bench_rccl_world1_under_torchrun(cuda):
    """The driver's multi-GPU command shape at N=1: torch.distributed.run, backend nccl (RCCL),
    eager communicator init bound to the device, reducer all-reduces and device barriers."""
    _run_rccl_world1([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                      "--master-addr", "127.0.0.1", "--master-port", str(free_port())], [])


def test_bench_rccl_world1_plain_python(cuda):
    """The driver's 1-GPU command (no launcher) joins a world-1 RCCL group too."""
    _run_rccl_world1([sys.executable], [])
