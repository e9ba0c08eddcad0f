"""The driver's bench.py contract, exercised on CPU/gloo with 2 ranks through
torch.distributed.run (tiny images): one JSON line from rank 0 with the
required keys, whole-job samples/s, max-over-ranks timing."""
import json
import os
import subprocess
import sys

import pytest

from dist_utils import free_port

pytestmark = pytest.mark.slow

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_py_two_ranks_cpu():
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--device", "cpu", "--batch", "2", "--image-size", "32"]
    env = dict(os.environ, OMP_NUM_THREADS="2", MADNN_LOG_LEVEL="WARNING")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in res
    assert res["n_gpus"] == 2 and res["steps"] == 2 and res["config"]["global_batch"] == 4
    assert res["config"]["parallelism"] == "dp2" and res["value"] > 0
    assert abs(res["value"] - 4 * 2 / (res["ms_per_step"] * 2 / 1000)) / res["value"] < 0.01


def test_launcher_tears_down_on_failure():
    code = ("import os,time,sys\n"
            "r=int(os.environ['RANK'])\n"
            "sys.exit(3) if r==1 else time.sleep(60)\n")
    script = os.path.join(ROOT, "gpurun_out", "_fail_script.py") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) \
        else "/tmp/_madnn_fail_script.py"
    with open(script, "w") as f:
        f.write(code)
    import time

    t0 = time.time()
    out = subprocess.run([sys.executable, "-m", "madnn.launch", "--nproc", "2", script], cwd=ROOT,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 3
    assert time.time() - t0 < 30  # rank 0 was torn down, not waited for
    os.remove(script)


def test_bench_py_gpt2_pipeline_four_ranks_cpu():
    """``bench.py --model gpt2-medium`` at 4 ranks = the 4-stage pipeline (first, two interior and
    last stage) of the BASELINE's GPT-2 PP config; short sequences, CPU/gloo."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "4", "--steps", "1", "--warmup", "1",
           "--device", "cpu", "--model", "gpt2-medium", "--batch", "4", "--seq-len", "32", "--microbatches", "4"]
    env = dict(os.environ, OMP_NUM_THREADS="1", MADNN_LOG_LEVEL="WARNING")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 4 and res["scaling"] == "strong" and res["value"] > 0
    assert res["config"]["parallelism"] == "pp4" and res["config"]["global_batch"] == 4
