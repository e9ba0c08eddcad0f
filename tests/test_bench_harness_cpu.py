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
           "--device", "cpu", "--batch", "2", "--image-size", "32", "--gpt2-config", "gpt2-tiny", "--seq-len", "32",
           "--gpt2-batch-per-gpu", "4", "--gpt2-mb", "2"]
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
    assert res["config"]["process_group"] == "gloo"
    # the automatic path and the numbers that explain an N > 1 result
    c = res["config"]
    # (on CPU the planner prices gloo against host compute: for 2 tiny images per rank it may
    # prefer a pipeline, which the bench records as rejected -- the metric is ResNet-50 DP)
    chosen = c["plan"] or c["plan_rejected"]
    assert chosen["comm_measured"] and chosen["dp"] * chosen["pp"] * chosen["tp"] == 2
    assert c["plan"] is None or c["plan"]["strategy"] == "dp"
    assert c["per_gpu_value"] == pytest.approx(res["value"] / 2, rel=1e-3)
    assert c["comm_exposed_ms"] is None or c["comm_exposed_ms"] >= 0
    assert c["p2p_gbps"] > 0 and c["probe_allreduce_busbw_gbps"] > 0
    assert "busbw_gbps" in c and c["tuning_timings"] == 0
    # the GPT-2 pipeline half of the BASELINE metric rides in the same line
    g = res["gpt2_pp"]
    assert g["parallelism"] == "pp2" and g["n_gpus"] == 2 and g["global_batch"] == 8 and g["microbatches"] == 4
    assert g["samples_per_s"] > 0 and g["tokens_per_s"] == pytest.approx(g["samples_per_s"] * 32, rel=1e-3)
    assert abs(g["samples_per_s"] - 8 * g["steps"] / (g["ms_per_step"] * g["steps"] / 1000)) / g["samples_per_s"] < 0.01
    assert g["loss_last_stage"] is None or g["loss_last_stage"] > 0


def test_bench_py_single_process_joins_world1_group():
    """No launcher: bench.py still creates a world-1 process group (gloo here, RCCL on the GPU)."""
    cmd = [sys.executable, "bench.py", "--steps", "1", "--warmup", "1", "--device", "cpu", "--batch", "2",
           "--image-size", "32", "--gpt2-config", "gpt2-tiny", "--seq-len", "16", "--gpt2-batch-per-gpu", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", MADNN_LOG_LEVEL="WARNING")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert res["n_gpus"] == 1 and res["config"]["process_group"] == "gloo"
    assert res["config"]["parallelism"] == "dp1" and res["gpt2_pp"]["parallelism"] == "dp1"
    assert res["ranks_seen"] == 1 and res["devices"] == ["cpu"]


def _no_launcher_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", MADNN_LOG_LEVEL="WARNING", **extra)
    return env


def test_bench_py_self_launches_n_ranks_without_launcher():
    """``bench.py --gpus 2`` with no launcher starts two ranks itself (the reference's one-command
    ``mpirun -n``, cifar_example/train.sh:14): the record says n_gpus 2 and the process group
    really had two ranks."""
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1", "--device", "cpu",
           "--model", "resnet50", "--batch", "2", "--std-batch", "0", "--image-size", "32", "--strategy", "dp"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=_no_launcher_env())
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["ranks_seen"] == 2 and len(res["devices"]) == 2
    assert res["config"]["parallelism"] == "dp2" and res["config"]["global_batch"] == 4


def test_bench_py_impossible_gpu_count_fails_loudly():
    """More ranks than devices (this container shows no GPU) must exit non-zero with the reason,
    never fall back to a smaller world."""
    cmd = [sys.executable, "bench.py", "--gpus", "4", "--steps", "1", "--warmup", "1", "--model", "resnet50"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300,
                         env=_no_launcher_env(HIP_VISIBLE_DEVICES="", CUDA_VISIBLE_DEVICES=""))
    assert out.returncode != 0
    assert "needs 4 visible devices" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_bench_py_launcher_world_mismatch_fails():
    """Under a launcher, a WORLD_SIZE that differs from --gpus is an error on every rank."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "4", "--steps", "1", "--warmup", "1",
           "--device", "cpu", "--model", "resnet50", "--batch", "2", "--image-size", "32"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert out.returncode != 0
    assert "WORLD_SIZE=2" in out.stderr


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
           "--device", "cpu", "--model", "gpt2-medium", "--gpt2-batch-per-gpu", "1", "--seq-len", "32",
           "--microbatches", "4"]
    env = dict(os.environ, OMP_NUM_THREADS="1", MADNN_LOG_LEVEL="WARNING")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 4 and res["scaling"] == "weak" and res["value"] > 0
    assert res["config"]["parallelism"] == "pp4" and res["config"]["global_batch"] == 4
    pp = res["gpt2_pp"]
    assert pp["microbatches"] == 4 and pp["model"] == "gpt2-medium"
    # the last stage's training and held-out losses reach rank 0's record
    assert pp["loss_last_stage"] > 0 and pp["heldout_loss"] > 0
    # the planner's choice and the transport numbers ride in the line
    assert pp["plan"]["pp"] == 4 and pp["plan"]["strategy"] == "pp" and pp["plan"]["comm_measured"]
    assert 0 < pp["bubble_fraction"] < 1 and pp["p2p_gbps"] > 0 and pp["p2p_bytes"] > 0
    assert pp["pp_plan"]["lags"][0] == 0.0 and pp["pp_plan"]["kept"] in pp["pp_plan"]["lags"]
    if len(pp["pp_plan"]["lags"]) > 1:   # both plans were timed before the warm-up
        assert len(pp["pp_plan"]["step_ms"]) == 2 and pp["plan_tuning_steps"] == 4


def _gpt2_8rank(extra_env=None, timeout=900, extra_args=()):
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "8", "--steps", "1", "--warmup", "1",
           "--device", "cpu", "--model", "gpt2-medium", "--gpt2-batch-per-gpu", "2", "--seq-len", "16",
           *extra_args]
    env = dict(os.environ, OMP_NUM_THREADS="1", MADNN_LOG_LEVEL="WARNING", **(extra_env or {}))
    return subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)


def test_bench_py_gpt2_dp2_pp4_interleaved_eight_ranks_emulated_rccl():
    """The 8-GPU layout of the GPT-2 half exactly as the driver's N=8 run builds it: GPT-2 medium,
    dp2 x pp4, interleaved 1F1B with 2 model chunks per rank (short sequences, CPU/gloo) -- with
    every point-to-point batch executed the way a fully serialising hardware queue would run it
    (``MADNN_EMULATE_RCCL_P2P``: rendezvous with complementary peer batches, host waits)."""
    out = _gpt2_8rank({"MADNN_EMULATE_RCCL_P2P": "1", "MADNN_EMULATE_RCCL_P2P_TIMEOUT": "120"},
                      extra_args=("--schedule", "interleaved", "--microbatches", "8"))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    pp = res["gpt2_pp"]
    assert res["n_gpus"] == 8 and res["value"] > 0 and "error" not in pp
    assert res["config"]["parallelism"] == "dp2xpp4"
    assert pp["schedule"] == "interleaved" and pp["virtual_stages"] in (2, 4) and pp["microbatches"] == 8


def test_bench_py_gpt2_eight_ranks_planner_schedule_emulated_rccl():
    """The default bench: the planner picks the schedule and microbatch count of the dp2 x pp4
    GPT-2 half (here from analytic costs), run under the emulated serialised transport."""
    out = _gpt2_8rank({"MADNN_EMULATE_RCCL_P2P": "1", "MADNN_EMULATE_RCCL_P2P_TIMEOUT": "120"})
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    pp = res["gpt2_pp"]
    assert "error" not in pp and res["config"]["parallelism"] == "dp2xpp4"
    assert pp["schedule"] in ("gpipe", "1f1b", "interleaved") and pp["planned_step_ms"] > 0
    assert 16 % pp["microbatches"] == 0


def test_bench_py_reports_resnet_when_gpt2_phase_fails():
    """The two halves are separate failure domains: a fault in the GPT-2 phase still prints the
    measured ResNet value (plus the standard-batch number) and exits non-zero."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--device", "cpu", "--batch", "4", "--std-batch", "2", "--image-size", "32", "--gpt2-config", "gpt2-tiny",
           "--seq-len", "16", "--gpt2-batch-per-gpu", "2", "--gpt2-mb", "1", "--gpt2-timeout", "60"]
    for fault in ("1:1:raise", "1:1:hang"):
        env = dict(os.environ, OMP_NUM_THREADS="2", MADNN_LOG_LEVEL="WARNING", MADNN_BENCH_GPT2_FAULT=fault)
        out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
        assert out.returncode != 0, fault
        lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
        assert len(lines) == 1, (fault, out.stdout, out.stderr[-2000:])
        res = json.loads(lines[0])
        assert res["value"] > 0 and res["config"]["parallelism"] == "dp2"
        assert res["config"]["std_batch"]["per_gpu_batch"] == 2 and res["config"]["std_batch"]["value"] > 0
        assert "error" in res["gpt2_pp"] and res["gpt2_pp"]["parallelism"] == "pp2", fault


@pytest.mark.parametrize("model,size", [("bert-large", "bert-tiny"), ("llama3-8b", "llama3-tiny")])
def test_bench_py_transformer_configs_two_ranks_cpu(model, size):
    """BASELINE configs 4 / 5 on the same timing contract: planner-chosen placement and
    checkpointing, the checkpointed-layer count and the plan in the record."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--device", "cpu", "--model", model, "--tf-config", size, "--seq-len", "32", "--tf-batch-per-gpu", "2"]
    env = dict(os.environ, OMP_NUM_THREADS="2", MADNN_LOG_LEVEL="WARNING")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    c = res["config"]
    assert res["unit"] == "tokens/s" and res["n_gpus"] == 2 and c["global_batch"] == 4 and c["seq_len"] == 32
    assert res["value"] == pytest.approx(4 * 32 * 2 / (res["ms_per_step"] * 2 / 1000), rel=1e-2)
    assert c["plan"]["dp"] * c["plan"]["pp"] * c["plan"]["tp"] == 2
    assert 0 <= c["checkpointed_layers"] <= c["layers"]
    # forward-only loss on a fresh batch, reported next to the training loss
    assert c["heldout_loss"] is not None and c["heldout_loss"] > 0 and c["ln_vocab"] > 0
