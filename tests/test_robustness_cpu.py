"""Robustness and plumbing (VERDICT r1 "dead hooks"):

* a hung rank turns into a process-group timeout and the launcher tears the job down,
  naming the failed rank (``madnn.launch --fault rank:step:hang``);
* a divergent collective order raises in ``verify_order`` (the engines call it every
  ``MADNN_CHECK_EVERY`` steps when ``check_collectives`` is on);
* the collective selector (R9) is the path ``synchronize_model`` takes;
* a launched world of ONE creates a real process group and the reducer issues its
  collectives (the 1-GPU rehearsal of the 8-GPU RCCL path);
* a second backward before the optimizer step is reduced too (no silently dropped grads);
* the stale-binary guard rejects a kernel library built from other sources.
"""
import copy
import json
import os
import shutil
import subprocess
import sys
import textwrap

import pytest
import torch
import torch.nn.functional as F

from dist_utils import free_port, run_dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ----------------------------------------------------------------- stale binary
def test_stale_binary_guard_detects_edited_source(tmp_path):
    from madnn.ops import build as b

    csrc = tmp_path / "csrc"
    shutil.copytree(b.CSRC, csrc)
    manifest = tmp_path / "manifest.json"
    b.write_manifest(csrc, manifest)
    assert b.stale_sources(csrc, manifest) == []
    src = csrc / "optim.hip"
    src.write_text(src.read_text() + "\n// edited\n")
    assert b.stale_sources(csrc, manifest) == ["optim.hip"]
    # a missing manifest means "unknown provenance": everything is stale
    assert "bucket.hip" in b.stale_sources(csrc, tmp_path / "none.json")


def test_shipped_kernel_library_matches_tree():
    from madnn.ops import build as b

    if not b.KERNELS_SO.exists():
        pytest.skip("kernel library not built")
    assert b.stale_sources() == [], "run `python -m madnn.ops.build`: the .so is stale"


def test_check_fresh_refuses_without_rebuild(tmp_path, monkeypatch):
    from madnn import ops
    from madnn.ops import build as b

    bad = tmp_path / "m.json"
    bad.write_text(json.dumps({"arch": b.ARCH, "sources": {"optim.hip": "0" * 16}}))
    monkeypatch.setattr(b, "MANIFEST", bad)
    monkeypatch.setattr(b.stale_sources, "__defaults__", (b.CSRC, bad))
    with pytest.raises(ops.StaleKernelsError, match="optim.hip"):
        ops.check_fresh(rebuild=False)


# ------------------------------------------------------------------- selector
def test_selector_paths_without_group():
    from madnn import comm

    sel = comm.select(torch.zeros(4), "all_reduce")
    assert sel.transport == "local" and sel.device == "cpu"
    assert sel(torch.zeros(4)) is None
    with pytest.raises(KeyError):
        comm.select(torch.zeros(1), "alltoall_bogus")


def _w_selector_and_sync(rank, world):
    import madnn
    from madnn import comm
    from madnn.models import MLP

    sel = comm.select(torch.zeros(2), "all_reduce")
    assert (sel.device, sel.transport, sel.mode) == ("cpu", "gloo", "sync")
    asel = comm.select(torch.zeros(2), "all_reduce", mode="async")
    t = torch.full((3,), float(rank + 1))
    work = asel(t, "sum")
    assert work is not None and work.wait()   # the async row returns a work handle
    torch.testing.assert_close(t, torch.full((3,), 3.0))
    table = comm.selector_table()
    assert table["cpu"]["singlenode"]["async"]["all_reduce"] == "gloo"
    assert set(table["cpu"]["singlenode"]) == {"sync", "async"}
    torch.manual_seed(rank)  # different replicas
    m = MLP(8, 16, 4)
    for p in m.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    madnn.synchronize_model(m)
    for p in m.parameters():
        torch.testing.assert_close(p.grad, torch.full_like(p, 1.5))
    flat = torch.cat([p.detach().flatten() for p in m.parameters()])
    allf = [torch.empty_like(flat) for _ in range(world)]
    torch.distributed.all_gather(allf, flat)
    torch.testing.assert_close(allf[0], allf[1], rtol=0, atol=0)


@pytest.mark.slow
def test_synchronize_model_via_selector_gloo():
    run_dist(_w_selector_and_sync, 2)


# ------------------------------------------------------------- order checker
def _w_order_diverges(rank, world):
    from madnn import comm

    comm.enable_order_check(True)
    t = torch.zeros(4 if rank == 0 else 8)  # same op count, different message: a schedule bug
    comm._record("all_reduce", None, t)
    with pytest.raises(RuntimeError, match="diverged"):
        comm.verify_order()


def _w_order_agrees(rank, world):
    import madnn
    from madnn import comm
    from madnn.models import MLP
    from madnn.optim import FusedSGD

    os.environ["MADNN_CHECK_EVERY"] = "2"
    torch.manual_seed(0)
    m = MLP(8, 16, 4)
    opt = FusedSGD(m.parameters(), lr=0.1)
    dm, opt = madnn.distribute(m, opt, strategy="dp", check_collectives=True)
    assert comm.order_check_enabled()
    for _ in range(4):  # verify_order runs inside after_step at steps 2 and 4
        F.cross_entropy(dm(torch.randn(4, 8)), torch.randint(4, (4,))).backward()
        opt.step()
    h, n = comm.order_fingerprint()
    assert n > 0
    comm.enable_order_check(False)


@pytest.mark.slow
def test_collective_order_divergence_raises():
    run_dist(_w_order_diverges, 2)


@pytest.mark.slow
def test_collective_order_check_in_engine_loop():
    run_dist(_w_order_agrees, 2)


# ------------------------------------------------------ hang -> timeout -> teardown
_HANG_SCRIPT = textwrap.dedent("""
    import sys, time
    sys.path.insert(0, {repo!r})
    import torch, torch.nn.functional as F
    import madnn
    from madnn.models import MLP
    from madnn.optim import FusedSGD
    madnn.init(device="cpu", timeout_s=6)
    torch.manual_seed(0)
    m = MLP(8, 16, 4)
    opt = FusedSGD(m.parameters(), lr=0.1)
    dm, opt = madnn.distribute(m, opt, strategy="dp", timeout_s=6)
    for step in range(6):
        F.cross_entropy(dm(torch.randn(4, 8)), torch.randint(4, (4,))).backward()
        opt.step()   # after_step -> maybe_fail(step): rank 1 hangs at step 2
    print("finished", flush=True)
""")


@pytest.mark.slow
def test_hung_rank_times_out_and_launcher_names_it(tmp_path):
    script = tmp_path / "hang.py"
    script.write_text(_HANG_SCRIPT.format(repo=REPO))
    env = dict(os.environ, MADNN_LOG_LEVEL="WARNING", OMP_NUM_THREADS="1")
    t = subprocess.run([sys.executable, "-m", "madnn.launch", "--nproc", "2", "--master-port", str(free_port()),
                        "--fault", "1:2:hang", "--timeout", "120", str(script)],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=180)
    assert t.returncode not in (0, 124), t.stderr[-3000:]   # failed, and not by the launcher's own timeout
    assert "rank 0 exited" in t.stderr, t.stderr[-3000:]    # the rank that saw the timeout is named
    assert "finished" not in t.stdout


def _w_monitored_barrier_names_rank(rank, world):
    from madnn import runtime as rt

    if rank == 1:
        import time

        time.sleep(8)
        return
    with pytest.raises(RuntimeError, match="1"):
        rt.barrier(timeout_s=2)


@pytest.mark.slow
def test_monitored_barrier_names_missing_rank():
    run_dist(_w_monitored_barrier_names_rank, 2)


# --------------------------------------------------------------- world of one
def _w_world1(rank, world):
    import torch.distributed as dist

    import madnn
    from madnn.models import MLP
    from madnn.optim import FusedSGD

    assert dist.is_initialized() and dist.get_world_size() == 1, "launched world-1 job must have a group"
    torch.manual_seed(0)
    m = MLP(8, 16, 4)
    ref = copy.deepcopy(m)
    opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.9)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    dm, opt = madnn.distribute(m, opt, strategy="dp", bucket_mb=0.0005)
    for _ in range(3):
        x, y = torch.randn(4, 8), torch.randint(4, (4,))
        F.cross_entropy(dm(x), y).backward()
        opt.step()
        ropt.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        ropt.step()
    assert dm.stats["buckets_launched"] >= 3 * len(dm.space.buckets)
    assert dm.stats["bytes_reduced"] > 0
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


@pytest.mark.slow
def test_launched_world_of_one_issues_collectives():
    run_dist(_w_world1, 1)


# ------------------------------------------------- two backwards, one step
def _w_double_backward(rank, world):
    import madnn
    from madnn.models import MLP
    from madnn.optim import FusedSGD

    torch.manual_seed(0)
    m = MLP(8, 16, 4)
    ref = copy.deepcopy(m)
    opt = FusedSGD(m.parameters(), lr=0.1)
    dm, opt = madnn.distribute(m, opt, strategy="dp")
    g = torch.Generator().manual_seed(7)
    xs = [torch.randn(2 * world, 8, generator=g) for _ in range(2)]
    ys = [torch.randint(4, (2 * world,), generator=g) for _ in range(2)]
    for x, y in zip(xs, ys):  # accumulation WITHOUT no_sync: each backward reduces
        F.cross_entropy(dm(x[2 * rank:2 * rank + 2]), y[2 * rank:2 * rank + 2]).backward()
    opt.step()
    assert dm.stats.get("rearmed", 0) == 1
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    for x, y in zip(xs, ys):
        F.cross_entropy(ref(x), y).backward()
    ropt.step()
    for p, q in zip(m.parameters(), ref.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


@pytest.mark.slow
def test_second_backward_before_step_is_reduced():
    run_dist(_w_double_backward, 2)


def _w_corrupt(rank, world, policy):
    """MADNN_FAULT=1:2:corrupt poisons rank 1's gradients of step 2 with NaN before the reduction;
    with nonfinite="skip" every rank skips that step together (weights stay finite and identical),
    with "raise" every rank raises NonFiniteGradients."""
    import os

    import madnn
    from madnn.models import MLP
    from madnn.optim import FusedSGD, NonFiniteGradients

    os.environ["MADNN_FAULT"] = "1:2:corrupt"
    torch.manual_seed(0)
    m = MLP(8, 16, 4)
    opt = FusedSGD(m.parameters(), lr=0.1)
    eng, opt = madnn.distribute(m, opt, strategy="dp", nonfinite=policy)
    x, y = torch.randn(4, 8), torch.randint(0, 4, (4,))
    snaps = []
    try:
        for _ in range(3):
            torch.nn.functional.cross_entropy(eng(x), y).backward()
            opt.step()
            snaps.append(torch.cat([p.detach().flatten().clone() for p in m.parameters()]))
    except NonFiniteGradients:
        assert policy == "raise" and len(snaps) == 1
        return
    assert policy == "skip" and opt.skipped_steps == 1
    assert all(torch.isfinite(s).all() for s in snaps)
    assert torch.equal(snaps[0], snaps[1]) and not torch.equal(snaps[1], snaps[2])  # step 2 skipped
    flat = snaps[-1]
    allf = [torch.empty_like(flat) for _ in range(world)]
    torch.distributed.all_gather(allf, flat)
    torch.testing.assert_close(allf[0], allf[1], rtol=0, atol=0)


@pytest.mark.slow
@pytest.mark.parametrize("policy", ["skip", "raise"])
def test_corrupt_gradients_skipped_or_raised_on_every_rank(policy):
    run_dist(_w_corrupt, 2, policy)


def _w_plan_measure(rank, world, fault_rank):
    import torch.distributed as dist

    from madnn.config import Config
    from madnn.planner import plan_model

    if fault_rank is not None:
        os.environ["MADNN_FAULT_MEASURE"] = str(fault_rank)
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.Tanh(), torch.nn.Linear(64, 64), torch.nn.Tanh(),
                                torch.nn.Linear(64, 4))
    cfg = Config.from_env(strategy="auto", measure=True, dtype="float32")
    plan = plan_model(model, cfg, world=world, example_input=torch.zeros(8, 16), global_batch=16)
    assert plan.measured == (fault_rank is None)
    # the measured links of this job priced the plan, identically on every rank
    assert plan.comm_probe["world"] == world and plan.comm_probe["p2p_gbps"] > 0
    mine = [(round(c.fwd_s, 12), round(c.bwd_s, 12)) for c in plan.costs] + [plan.describe()]
    got = [None] * world
    dist.all_gather_object(got, mine)
    assert all(g == got[0] for g in got)


@pytest.mark.parametrize("fault_rank", [None, 1, 0])
def test_planner_measurement_failure_is_agreed_not_hung(fault_rank):
    """One rank's layer timing raising (MADNN_FAULT_MEASURE) makes EVERY rank fall back to the
    analytic costs -- no rank is left blocked in the results all-gather -- and all ranks plan the
    same placement; without a fault the CPU timings are used."""
    run_dist(_w_plan_measure, 2, fault_rank)


def _w_local_groups(rank, world):
    import torch.distributed as dist

    import madnn
    from madnn import comm
    from madnn import runtime as rt

    groups = rt.ProcessGroups(rt.Mesh(dp=world, pp=1, tp=1))
    # size-one axes get no communicator (no RCCL stream); the dp axis spans the world
    for g in (groups.pp_group, groups.tp_group, groups.cp_group):
        assert isinstance(g, rt.LocalGroup) and rt.get_world_size(g) == 1 and rt.get_rank(g) == 0
    assert groups.dp_group is None
    t = torch.full((3,), float(rank + 1))
    assert comm.all_reduce(t, "sum", group=groups.pp_group) is None and t.eq(rank + 1).all()
    assert comm.select(t, "all_reduce", groups.tp_group).transport == "local"
    rt.barrier(groups.cp_group)
    assert comm.verify_order(groups.pp_group)
    comm.all_reduce(t, "sum", group=groups.dp_group)
    assert t.eq(sum(range(1, world + 1))).all()
    assert dist.get_world_size() == world


def test_singleton_axes_create_no_process_group():
    run_dist(_w_local_groups, 2)


def _w_agreed_budget(rank, world):
    from madnn.planner import _agreed_min

    # ranks holding different amounts of memory: every rank sees the tightest budget, so the
    # chain calibration takes the same early return / the same chain batch on all of them
    assert _agreed_min(1e9 if rank == 0 else -5.0) == -5.0
    assert _agreed_min(float(10 + rank)) == 10.0


def test_chain_calibration_budget_is_agreed_across_ranks():
    run_dist(_w_agreed_budget, 2)
