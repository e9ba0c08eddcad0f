"""T0: single-process unit tests (no GPU, no process group).

Reference semantics pinned here: contiguous striping with the remainder
dropped (datamodule.lua:239-246), the sync-period heuristic
(datamodule.lua:68-78), parallelize's usage/-1 return (:18-21); plus the C++
runtime (partitioner, bucket planner, pipeline programs), planner decisions,
tracer, cost model, fused optimizers vs torch.optim, config precedence.
"""
import math
import os

import pytest
import torch
import torch.nn.functional as F
from torch import nn

import madnn
from madnn import ops
from madnn.config import Config
from madnn.data import DistributedSampler, shard, shard_bounds
from madnn.ops import native_runtime as nr
from madnn.parallel.dp import default_sync_period


# ------------------------------------------------------------------ data (R5)
def test_shard_contiguous_remainder_dropped():
    data = torch.arange(10)
    parts = [shard(data, r, 3) for r in range(3)]
    assert [p.tolist() for p in parts] == [[0, 1, 2], [3, 4, 5], [6, 7, 8]]  # sample 9 dropped (reference)
    assert parts[0].data_ptr() == data.data_ptr()  # a view, like the reference's data[{{s,e}}]


def test_shard_remainder_policies():
    assert shard_bounds(10, 2, 3, "last") == (6, 10)
    padded = [shard(torch.arange(10), r, 3, remainder="pad").tolist() for r in range(3)]
    assert set(sum(padded, [])) == set(range(10))  # every sample seen, wrap-around pads
    assert all(len(p) == 4 for p in padded)
    assert shard(torch.arange(10), 1, 3, strided=True).tolist() == [1, 4, 7]


def test_sampler_covers_shard_and_shuffles():
    s = DistributedSampler(100, rank=1, world=4, shuffle=True, seed=3)
    idx = list(iter(s))
    assert sorted(idx) == list(range(25, 50))
    s.set_epoch(1)
    assert list(iter(s)) != idx


# ----------------------------------------------------------- sync period (R6)
@pytest.mark.parametrize("n,k", [(10, 1), (999, 1), (1000, 10), (2499, 10), (2500, 50), (4999, 50), (5000, 100)])
def test_sync_period_heuristic(n, k):
    assert default_sync_period(n) == k


def test_parallelize_usage_returns_minus_one(capsys):
    assert madnn.parallelize(None, torch.zeros(3), nn.Linear(2, 2)) == -1
    assert "usage" in capsys.readouterr().out


def test_parallelize_single_process():
    m = nn.Linear(4, 2)
    d, t, n = madnn.parallelize(torch.randn(10, 4), torch.zeros(10), m, verbose=False)
    assert n == 10 and m._madnn_sync.period == 1
    d, t, n = madnn.parallelize(torch.randn(10, 4), torch.zeros(10), m, sync_every=-1, verbose=False)
    assert m._madnn_sync is None


# ------------------------------------------------------------ native runtime
def test_partition_minimises_bottleneck():
    bounds, best = nr.partition([1, 1, 1, 1, 4, 1, 1, 1], 3)
    assert bounds[0] == 0 and bounds[-1] == 8 and len(bounds) == 4
    stages = [sum([1, 1, 1, 1, 4, 1, 1, 1][bounds[i]:bounds[i + 1]]) for i in range(3)]
    assert max(stages) == best == 4


def test_partition_memory_cap():
    with pytest.raises(ValueError):
        nr.partition([1, 1, 1], 2, mems=[10, 10, 10], mem_cap=15)
    b, _ = nr.partition([1, 1, 1, 1], 2, mems=[1, 1, 10, 1], mem_cap=11)
    assert b == [0, 2, 4]


def test_plan_buckets_alignment_and_cap():
    bo, oo, bs = nr.plan_buckets([10, 20, 5, 100, 3], cap_elems=64, align=16)
    assert bo == [0, 0, 0, 1, 2]
    assert oo == [0, 16, 48, 0, 0]
    assert all(o % 16 == 0 for o in oo)
    assert bs == [64, 112, 16]


@pytest.mark.parametrize("kind,V", [("gpipe", 1), ("1f1b", 1), ("interleaved", 2), ("interleaved", 3)])
@pytest.mark.parametrize("S,M", [(2, 4), (4, 4), (4, 8), (3, 6), (2, 2)])
def test_pipeline_orders_deadlock_free_and_fifo(kind, V, S, M):
    """Every rank's compute order against one-directional FIFO channels with non-blocking
    sends: no deadlock, each channel received in send order (what lets the engine post all
    receives up front), every (chunk, microbatch) forward and backward exactly once."""
    from madnn.parallel.pp import simulate_schedule

    for s in range(S):
        order = nr.pipeline_order(kind, s, S, M, V)
        for op in ("F", "B"):
            assert sorted((c, m) for o, c, m in order if o == op) == [(c, m) for c in range(V) for m in range(M)]
    r = simulate_schedule(kind, S, M, V)
    if kind == "1f1b":
        assert r["peak_inflight"] == [min(S - s, M) for s in range(S)]
        assert r["bubble"] == pytest.approx((S - 1) / (M + S - 1), abs=1e-9)


_PLANS = [(k, V, S, M) for S in (2, 4, 8) for k, V in (("gpipe", 1), ("1f1b", 1), ("interleaved", 2))
          for M in sorted({S, 8, 16, 32}) if k != "interleaved" or M % S == 0]


@pytest.mark.parametrize("lag", [0.0, 0.3])
@pytest.mark.parametrize("kind,V,S,M", _PLANS)
def test_issue_plan_messages_pair_up_fifo(kind, V, S, M, lag):
    """Every message of every rank's issue plan is sent once and received once, in the same order
    on both ends of each rank pair, and every compute's input comes from a batch before it --
    for both plans the engine can run (boundaries on the compute-only clock, lag 0, and on a
    clock with transfers 0.3 of a forward long)."""
    from madnn.parallel.pp import check_plan_fifo, issue_plan

    assert check_plan_fifo(kind, S, M, V, lag) == 2 * M * (S * V - 1)
    for s in range(S):
        have = set()
        for item in issue_plan(kind, s, S, M, V, lag):
            if item[0] == "X":
                assert 1 <= len(item[1]) <= 4
                have |= {(k, c, m) for d, k, c, m, _p in item[1] if d == "recv"}
            else:
                _, op, c, m = item
                vs = c * S + s
                if op == "F" and vs > 0:
                    assert ("act", c, m) in have
                if op == "B" and vs < S * V - 1:
                    assert ("grad", c, m) in have


@pytest.mark.parametrize("lag", [0.0, 0.3])
@pytest.mark.parametrize("kind,V,S,M", _PLANS)
def test_pipeline_transport_safe_under_hw_queue_sharing(kind, V, S, M, lag):
    """The engine's program (issue_plan on the act/grad communicators, DP all-reduce, tied sum)
    completes when every stream of a rank feeds ONE serialising hardware queue, on any rotation of
    a 4-queue (HIP's GPU_MAX_HW_QUEUES default) and a 2-queue round-robin pool, and with
    independent queues -- dp1 and dp2 meshes, steady state and the first step's host-blocking
    shape headers, for both issue plans the engine chooses between (lag 0 and 0.3)."""
    from madnn.parallel.pp import simulate_schedule, simulate_transport

    for dp in (1, 2):
        for first in (False, True):
            for q, offs in (("serial", [0]), (4, range(4)), (2, range(2)), (None, [0])):
                for off in offs:
                    simulate_transport(kind, S, M, V, "split", q, dp=dp, tied=True, first_step=first,
                                       queue_offset=off, t_p2p=lag / 2, lag=lag)
    # with free transfers the transport adds no bubble over the compute-only schedule
    r = simulate_transport(kind, S, M, V, "split", None, lag=lag)
    assert r["bubble"] == pytest.approx(simulate_schedule(kind, S, M, V)["bubble"], abs=1e-9)


@pytest.mark.parametrize("kind,V,S,M", [("gpipe", 1, 2, 8), ("1f1b", 1, 3, 8), ("1f1b", 1, 4, 16),
                                        ("interleaved", 2, 4, 16), ("1f1b", 1, 8, 32)])
def test_round3_preposted_receives_deadlock_when_queues_serialise(kind, V, S, M):
    """The round-3 transport (one 2-rank communicator per channel, every receive of the step posted
    before the first compute) is fine with independent queues but deadlocks once a rank's streams
    share one serialising queue; at pp >= 4 with dp2 it deadlocks on EVERY rotation of the default
    4-queue pool -- the driver's dp2 x pp4 GPT-2 layout."""
    from madnn.parallel.pp import simulate_transport

    simulate_transport(kind, S, M, V, "prepost", None)
    with pytest.raises(RuntimeError, match="deadlocks"):
        simulate_transport(kind, S, M, V, "prepost", "serial")
    if S >= 4 and kind != "gpipe":
        for off in range(4):
            with pytest.raises(RuntimeError, match="deadlocks"):
                simulate_transport(kind, S, M, V, "prepost", 4, dp=2, tied=True, queue_offset=off)


def test_split_transport_keeps_1f1b_transfers_off_the_critical_path():
    """With real transfer times (a quarter of a microbatch forward) the engine's act/grad split
    prices 1F1B exactly like the unsafe round-3 pre-posting, and beats one shared communicator."""
    from madnn.parallel.pp import simulate_transport

    for S in (4, 8):
        split = simulate_transport("1f1b", S, 16, 1, "split", None, dp=2, tied=True, t_p2p=0.25)["makespan"]
        one = simulate_transport("1f1b", S, 16, 1, "batched", None, dp=2, tied=True, t_p2p=0.25)["makespan"]
        pre = simulate_transport("1f1b", S, 16, 1, "prepost", None, dp=2, tied=True, t_p2p=0.25)["makespan"]
        assert split == pytest.approx(pre) and split < one


def test_interleaving_shrinks_the_bubble():
    from madnn.parallel.pp import pipeline_bubble

    b1 = pipeline_bubble("1f1b", 4, 16, 1)
    b2 = pipeline_bubble("interleaved", 4, 16, 2)
    b3 = pipeline_bubble("interleaved", 4, 16, 3)
    assert b1 == pytest.approx(3 / 19)
    assert b3 < b2 < b1 and b2 < 0.6 * b1


def test_pipeline_order_rejects_bad_interleave():
    with pytest.raises(ValueError):
        nr.pipeline_order("interleaved", 0, 4, 6, 2)  # M % S != 0
    with pytest.raises(ValueError):
        nr.pipeline_order("1f1b", 0, 4, 8, 2)


def test_order_hash():
    a, b = nr.OrderHash(), nr.OrderHash()
    for h in (a, b):
        h.add(1, 0, 100, 1)
        h.add(2, 3, 7, 0)
    assert a.h == b.h and a.count == 2
    b.add(1, 0, 1, 1)
    assert a.h != b.h


# -------------------------------------------------------------------- config
def test_config_env_precedence(monkeypatch):
    monkeypatch.setenv("MADNN_BUCKET_MB", "12.5")
    monkeypatch.setenv("MADNN_SYNC", "params")
    c = Config.from_env()
    assert c.bucket_mb == 12.5 and c.sync == "params"
    c = Config.from_env(bucket_mb=3.0)
    assert c.bucket_mb == 3.0
    with pytest.raises(ValueError):
        Config.from_env(strategy="bogus")


# -------------------------------------------------------- fused optimizers (CPU)
@pytest.mark.parametrize("kind", ["sgd", "adamw", "adam_l2"])
def test_fused_optimizer_standalone_matches_torch(kind):
    from madnn.optim import FusedAdam, FusedSGD

    torch.manual_seed(0)
    m1 = nn.Sequential(nn.Linear(8, 16), nn.Tanh(), nn.Linear(16, 3))
    m2 = nn.Sequential(nn.Linear(8, 16), nn.Tanh(), nn.Linear(16, 3))
    m2.load_state_dict(m1.state_dict())
    if kind == "sgd":
        o1 = FusedSGD([{"params": m1[0].parameters(), "lr": 0.05}, {"params": m1[2].parameters()}], lr=0.1,
                      momentum=0.9, nesterov=True, weight_decay=1e-3)
        o2 = torch.optim.SGD([{"params": m2[0].parameters(), "lr": 0.05}, {"params": m2[2].parameters()}], lr=0.1,
                             momentum=0.9, nesterov=True, weight_decay=1e-3)
    elif kind == "adamw":
        o1 = FusedAdam(m1.parameters(), lr=1e-2, weight_decay=0.1, adamw=True)
        o2 = torch.optim.AdamW(m2.parameters(), lr=1e-2, weight_decay=0.1)
    else:
        o1 = FusedAdam(m1.parameters(), lr=1e-2, weight_decay=0.1, adamw=False)
        o2 = torch.optim.Adam(m2.parameters(), lr=1e-2, weight_decay=0.1)
    s1 = torch.optim.lr_scheduler.StepLR(o1, 2, 0.5)
    s2 = torch.optim.lr_scheduler.StepLR(o2, 2, 0.5)
    x, y = torch.randn(32, 8), torch.randint(0, 3, (32,))
    for _ in range(5):
        for m, o, s in ((m1, o1, s1), (m2, o2, s2)):
            o.zero_grad()
            F.cross_entropy(m(x), y).backward()
            o.step()
            s.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)
    sd = o1.state_dict()
    st2 = o2.state_dict()["state"]
    key = "momentum_buffer" if kind == "sgd" else "exp_avg"
    torch.testing.assert_close(sd["state"][0][key], st2[0][key], atol=1e-5, rtol=1e-5)


def test_fused_clip_grad_norm_matches_torch():
    from madnn.optim import FusedSGD

    torch.manual_seed(1)
    m1, m2 = nn.Linear(10, 10), nn.Linear(10, 10)
    m2.load_state_dict(m1.state_dict())
    o1, o2 = FusedSGD(m1.parameters(), lr=0.1), torch.optim.SGD(m2.parameters(), lr=0.1)
    x = torch.randn(4, 10) * 10
    m1(x).pow(2).sum().backward()
    m2(x).pow(2).sum().backward()
    n1 = o1.clip_grad_norm_(0.5)
    n2 = torch.nn.utils.clip_grad_norm_(m2.parameters(), 0.5)
    assert abs(float(n1) - float(n2)) < 1e-3 * float(n2)
    o1.step()
    o2.step()
    torch.testing.assert_close(m1.weight, m2.weight, atol=1e-5, rtol=1e-5)


# ------------------------------------------------------ tracer / cost / planner
def test_fx_spine_composes_to_model():
    from madnn.models import resnet18
    from madnn.planner.trace import run_spine, trace

    from madnn.planner.trace import _fx_split

    m = resnet18(num_classes=7).eval()
    x = torch.randn(2, 3, 64, 64)
    sp = _fx_split(m)  # the fx path on its own (ResNet also declares its spine)
    assert sp.source == "fx" and len(sp) > 5
    torch.testing.assert_close(run_spine(sp, x), m(x))
    sp = trace(m)
    assert sp.source == "declared" and len(sp) == 2 + 8
    torch.testing.assert_close(run_spine(sp, x), m(x))


def test_fx_spine_resnet50_bottleneck_fusions():
    """ResNet-50's bottlenecks (dual downsample BN, bn -> conv fusions) stay fx-traceable: the fused
    paths are skipped for proxies and the spine still composes to the model."""
    from madnn.models import resnet50
    from madnn.planner.trace import _fx_split, run_spine

    m = resnet50(num_classes=7).eval()
    sp = _fx_split(m)
    assert sp is not None and sp.source == "fx" and len(sp) > 16
    x = torch.randn(2, 3, 64, 64)
    torch.testing.assert_close(run_spine(sp, x), m(x))


def test_declared_spine_and_block_list():
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.planner.trace import run_spine, trace

    m = GPT2(gpt2_config("gpt2-tiny")).eval()
    sp = trace(m)
    assert sp.source == "declared" and sp.block_list == "h" and len(sp) == 6
    ids = torch.randint(0, 512, (2, 16))
    torch.testing.assert_close(run_spine(sp, ids), m(ids))


def test_cost_model_flops_gpt2():
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.planner import estimate, trace

    with torch.device("meta"):
        m = GPT2(gpt2_config("gpt2-medium"))
    costs = estimate(trace(m), torch.zeros(1, 1024, dtype=torch.long))
    flops = sum(c.flops for c in costs)
    n = sum(p.numel() for p in m.parameters())
    # forward ~ 2 FLOPs per parameter per token (+ attention), 1024 tokens
    assert 2 * n * 1024 * 0.9 < flops < 2 * n * 1024 * 1.6
    assert costs[0].params > 50e6 and costs[-1].shared_params > 50e6  # tied wte/lm_head detected


def test_planner_choices():
    from madnn.models.llama import Llama, llama_config
    from madnn.planner import plan_model

    with torch.device("meta"):
        m = Llama(llama_config("llama3-8b"))
    ex = torch.zeros(1, 4096, dtype=torch.long)
    p = plan_model(m, Config.from_env(strategy="auto", global_batch=64), 8, example_input=ex)
    assert p.dp * p.pp * p.tp == 8 and max(p.est_mem_gb) <= 288 * 0.85
    p = plan_model(m, Config.from_env(strategy="pp", pp_stages=4, global_batch=64), 4, example_input=ex)
    assert (p.dp, p.pp) == (1, 4) and p.bounds[0] == 0 and p.bounds[-1] == 34
    p = plan_model(m, Config.from_env(strategy="dp_pp", pp_stages=2, global_batch=64), 8, example_input=ex)
    assert (p.dp, p.pp) == (4, 2)


def test_planner_ws8_table_covers_all_strategies():
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.planner import plan_model

    with torch.device("meta"):
        m = GPT2(gpt2_config("gpt2-medium"))
    ex = torch.zeros(1, 1024, dtype=torch.long)
    p = plan_model(m, Config.from_env(strategy="auto", global_batch=128), 8, example_input=ex)
    kinds = {c["strategy"] for c in p.candidates}
    assert kinds >= {"dp", "pp", "dp_pp", "tp"}, kinds
    assert "| tp |" in p.table() and "| dp_pp |" in p.table()
    assert not p.measured  # no GPU here: analytic costs


def test_planner_interleaved_plan_shape():
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.planner import plan_model

    with torch.device("meta"):
        m = GPT2(gpt2_config("gpt2-medium"))
    ex = torch.zeros(1, 1024, dtype=torch.long)
    p = plan_model(m, Config.from_env(strategy="pp", pp_stages=4, schedule="interleaved", global_batch=64), 4,
                   example_input=ex)
    assert p.virtual in (2, 4) and p.schedule == "interleaved" and len(p.bounds) == 4 * p.virtual + 1
    assert p.microbatches % 4 == 0
    q = plan_model(m, Config.from_env(strategy="pp", pp_stages=4, schedule="1f1b", global_batch=64), 4,
                   example_input=ex)
    # same work, smaller bubble
    assert p.est_step_s < q.est_step_s
    v2 = plan_model(m, Config.from_env(strategy="pp", pp_stages=4, schedule="interleaved", virtual_stages=2,
                                       microbatches=16, global_batch=64), 4, example_input=ex)
    assert (v2.virtual, v2.microbatches) == (2, 16)


def test_planner_searches_schedules_and_microbatches():
    """schedule="auto" (the default): every PP row of the table is one (schedule, V, M) variant --
    GPipe, 1F1B and interleaved with 2 and 4 chunks at several microbatch counts -- and the
    chosen one is the cheapest feasible row."""
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.planner import plan_model

    with torch.device("meta"):
        m = GPT2(gpt2_config("gpt2-medium"))
    ex = torch.zeros(1, 1024, dtype=torch.long)
    p = plan_model(m, Config.from_env(strategy="pp", pp_stages=4, global_batch=64), 4, example_input=ex)
    rows = {(c["schedule"], c["V"], c["M"]) for c in p.candidates}
    assert {"gpipe", "1f1b", "interleaved"} <= {r[0] for r in rows}
    assert {2, 4} <= {r[1] for r in rows if r[0] == "interleaved"}
    assert {4, 8, 16} <= {r[2] for r in rows if r[0] == "1f1b"}
    assert "| interleaved V=2 |" in p.table() and "| interleaved V=4 |" in p.table()
    best = min((c for c in p.candidates if c["fits"]), key=lambda c: c["step_s"])
    assert (p.schedule, p.virtual, p.microbatches) == (best["schedule"], best["V"], best["M"])
    # per-call fixed costs make tiny microbatches expensive: the search does not just max out M
    assert all(c["step_s"] > 0 for c in p.candidates)


def test_planner_auto_pipeline_when_a_replica_does_not_fit():
    """Automatic placement picks a pipeline when no data-parallel replica fits one GPU: Llama-3
    70B (~1.1 TB of mixed-precision Adam state) at 8 GPUs becomes pp=8 with checkpointing and the
    cheapest schedule, every stage inside 288 GB; the DP rows are all marked as not fitting."""
    from madnn.models.llama import Llama, llama_config
    from madnn.planner import plan_model

    with torch.device("meta"):
        m = Llama(llama_config("llama3-70b"))
    p = plan_model(m, Config.from_env(strategy="auto"), 8, example_input=torch.zeros(1, 2048, dtype=torch.long),
                   global_batch=32)
    assert (p.strategy, p.dp, p.pp) == ("pp", 1, 8), p.describe()
    assert max(p.est_mem_gb) <= 309.3 * 0.85 and any(p.checkpoint)
    assert all(not c["fits"] for c in p.candidates if c["strategy"] == "dp")
    assert "V=" in p.table() or p.virtual == 1


def test_planner_checkpoints_the_fewest_blocks_that_fit():
    """Per-block activation checkpointing: Llama-3 8B at 8192 tokens x 4 sequences on one GPU does
    not fit without recompute and does not need it on every block.  The planner prices no
    recompute, every block, and the per-block choice, and takes the per-block plan: 0 < k < 32
    blocks, inside the HBM cap, faster than recomputing all of them (the reference's analog is its
    size-driven automatic knob, datamodule.lua:65-78)."""
    from madnn.models.llama import Llama, llama_config
    from madnn.planner import plan_model

    with torch.device("meta"):
        m = Llama(llama_config("llama3-8b"))
    p = plan_model(m, Config.from_env(strategy="auto", checkpointing="auto"), 1,
                   example_input=torch.zeros(1, 8192, dtype=torch.long), global_batch=4)
    k = sum(p.checkpoint)
    assert 0 < k < 32, p.describe()
    assert not p.checkpoint[0] and not p.checkpoint[-1]          # embedding and head never recomputed
    rows = {c["ckpt"]: c for c in p.candidates}
    assert not rows[0]["fits"] and rows[32]["fits"] and rows[k]["fits"]
    assert rows[k]["step_s"] < rows[32]["step_s"] and p.est_step_s == rows[k]["step_s"]
    # a smaller problem fits without any recompute: the knob follows the problem size
    p2 = plan_model(m, Config.from_env(strategy="auto", checkpointing="auto"), 1,
                    example_input=torch.zeros(1, 1024, dtype=torch.long), global_batch=4)
    assert sum(p2.checkpoint) == 0


def test_measured_costs_change_the_placement():
    """The planner consumes measured layer times: with GPT-2 medium at 8 GPUs, analytic costs
    and costs that make compute 100x cheaper (comm-dominated) must not pick the same layout,
    and skewed per-layer measurements move the pipeline stage boundaries."""
    import copy

    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.planner import estimate, plan_model, trace

    with torch.device("meta"):
        m = GPT2(gpt2_config("gpt2-medium"))
    ex = torch.zeros(1, 1024, dtype=torch.long)
    cfg = Config.from_env(strategy="auto", global_batch=16)
    base = estimate(trace(m), ex)
    p0 = plan_model(m, cfg, 8, example_input=ex, costs=copy.deepcopy(base))
    fast = copy.deepcopy(base)
    for c in fast:
        c.fwd_s, c.bwd_s, c.fixed_s, c.measured = c.fwd_s / 100, c.bwd_s / 100, c.fixed_s / 100, True
    p1 = plan_model(m, cfg, 8, example_input=ex, costs=fast)
    assert p1.measured and not p0.measured
    assert (p0.strategy, p0.dp, p0.pp, p0.tp) != (p1.strategy, p1.dp, p1.pp, p1.tp)
    cfg_pp = Config.from_env(strategy="pp", pp_stages=4, schedule="1f1b", microbatches=8, global_batch=64)
    q0 = plan_model(m, cfg_pp, 4, example_input=ex, costs=copy.deepcopy(base))
    skew = copy.deepcopy(base)
    for c in skew[1:6]:  # the first blocks measure 3x slower than the model says
        c.fwd_s, c.bwd_s, c.measured = c.fwd_s * 3, c.bwd_s * 3, True
    q1 = plan_model(m, cfg_pp, 4, example_input=ex, costs=skew)
    assert q1.bounds != q0.bounds and q1.bounds[1] < q0.bounds[1]


def test_dp_exposed_timeline():
    from madnn.planner import dp_exposed_s
    from madnn.planner.hw import Machine

    hw = Machine()
    mb = 64 * 2**20
    ar = hw.allreduce_s(mb, 8)
    # all gradients land at the very end (one layer): the whole reduction is exposed
    assert dp_exposed_s([1e-3], [mb], 8, hw, mb) == pytest.approx(ar)
    # ten equal layers, one bucket each, backward much longer than a reduction: only the last
    exp = dp_exposed_s([10 * ar] * 10, [mb] * 10, 8, hw, mb)
    assert exp == pytest.approx(ar)
    # comm-bound: reductions queue up behind each other
    exp = dp_exposed_s([ar / 10] * 10, [mb] * 10, 8, hw, mb)
    assert exp == pytest.approx(10 * ar - 9 * ar / 10, rel=1e-6)
    assert dp_exposed_s([1.0], [mb], 1, hw, mb) == 0.0


def test_hw_profile_precedence(tmp_path, monkeypatch):
    import json as _json

    from madnn.planner import hw

    prof = tmp_path / "p.json"
    prof.write_text(_json.dumps({"hbm_tbps": 4.2, "bf16_tflops": 901.0, "calibrated": "test"}))
    monkeypatch.setenv("MADNN_HW_PROFILE", str(prof))
    hw.invalidate()
    m = hw.load()
    assert m.hbm_tbps == 4.2 and m.bf16_tflops == 901.0 and m.source == str(prof)
    monkeypatch.delenv("MADNN_HW_PROFILE")
    hw.invalidate()
    assert hw.load().source in (hw.default_profile_path(), hw.SHIPPED, "defaults")


# ---------------------------------------------------------------- nn modules
def test_fused_layernorm_cpu_matches_torch_and_swap():
    from madnn.nn import FusedLayerNorm, swap_layernorms

    ln = nn.LayerNorm(64)
    nn.init.normal_(ln.weight)
    f = FusedLayerNorm(64)
    f.load_state_dict(ln.state_dict())
    x = torch.randn(3, 5, 64)
    torch.testing.assert_close(f(x), ln(x), atol=1e-5, rtol=1e-5)
    seq = nn.Sequential(nn.Linear(64, 64), nn.LayerNorm(64))
    ref = seq(x)
    assert swap_layernorms(seq) == 1 and isinstance(seq[1], FusedLayerNorm)
    torch.testing.assert_close(seq(x), ref, atol=1e-5, rtol=1e-5)


def test_fused_batchnorm_cpu_path_is_eager():
    from madnn.nn import FusedBatchNorm2d

    bn, ref = FusedBatchNorm2d(8), nn.BatchNorm2d(8)
    x, r = torch.randn(4, 8, 5, 5), torch.randn(4, 8, 5, 5)
    torch.testing.assert_close(bn(x, residual=r, relu=True), torch.relu(ref(x) + r))
    torch.testing.assert_close(bn.running_mean, ref.running_mean)
    assert int(bn.num_batches_tracked) == 1


def test_mp_layers_world_of_one_equal_dense():
    import madnn.nn as mnn

    torch.manual_seed(0)
    d1, d2 = nn.Linear(16, 32), nn.Linear(32, 4)
    mp = nn.Sequential(mnn.MPInitialReshape(16), mnn.MPInitialLinear(16, 32), mnn.MPTanh(), mnn.MPBaseLinear(32, 4))
    mp[1].load_full(d1.weight, d1.bias)
    mp[3].load_full(d2.weight, d2.bias)
    x = torch.randn(3, 4, 4)
    torch.testing.assert_close(mp(x), d2(torch.tanh(d1(x.reshape(3, 16)))))


def test_synthetic_batch_deterministic():
    a = madnn.data.synthetic_batch("tokens", 2, "cpu", seq_len=8, vocab=100, seed=3)[0]
    b = madnn.data.synthetic_batch("tokens", 2, "cpu", seq_len=8, vocab=100, seed=3)[0]
    assert torch.equal(a, b)


def test_fault_injection_parse():
    from madnn.utils import fault

    os.environ["MADNN_FAULT"] = "0:3:raise"
    try:
        fault.maybe_fail(2, rank=0)
        with pytest.raises(fault.InjectedFault):
            fault.maybe_fail(3, rank=0)
        fault.maybe_fail(3, rank=1)
    finally:
        del os.environ["MADNN_FAULT"]


def test_kernel_library_built_for_gfx950(tmp_path):
    """build() output exists and carries a gfx950 code object (checked without a GPU; the bundles are
    extracted next to a copy in tmp_path, never beside the in-tree library)."""
    import shutil
    import subprocess

    so = ops.kernels_path()
    if not so.exists():
        pytest.skip("kernel library not built")
    local = tmp_path / so.name
    shutil.copy(so, local)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(local)], capture_output=True,
                         text=True)
    assert "gfx950" in out.stdout + out.stderr


def test_miopen_find_db_seeding(tmp_path, monkeypatch):
    """setup_find_db copies the shipped MI355X find/perf dbs into a writable dir and exports
    MIOPEN_USER_DB_PATH, but never overrides a path the user already set."""
    from madnn.utils import miopen

    shipped = sorted(p.name for p in miopen.SHIPPED_DB.iterdir() if p.name.endswith(".txt"))
    assert any(n.endswith(".ufdb.txt") for n in shipped) and any(n.endswith(".udb.txt") for n in shipped)
    monkeypatch.delenv("MIOPEN_USER_DB_PATH", raising=False)
    got = miopen.setup_find_db(workdir=tmp_path / "db")
    assert got == str(tmp_path / "db") and sorted(p.name for p in (tmp_path / "db").iterdir()) == shipped
    monkeypatch.setenv("MIOPEN_USER_DB_PATH", "/somewhere/else")
    assert miopen.setup_find_db() == "/somewhere/else"


def test_distribute_meta_model_remaps_optimizer():
    """A model built on the meta device (with its optimizer) is materialised by distribute(dp)
    and the optimizer steps the real parameters."""
    import madnn
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.optim import FusedAdam

    torch.manual_seed(0)
    with torch.device("meta"):
        model = GPT2(gpt2_config("gpt2-tiny"))
    opt = FusedAdam(model.parameters(), lr=1e-3)
    eng, opt = madnn.distribute(model, opt, strategy="dp")
    assert not any(p.is_meta for g in opt.param_groups for p in g["params"])
    ids = torch.randint(0, model.config.vocab_size, (2, 16))
    before = [p.detach().clone() for p in model.parameters()]
    loss = eng.train_step(ids, ids)
    opt.step()
    assert torch.isfinite(loss)
    assert any(not torch.equal(b, p.detach()) for b, p in zip(before, model.parameters()))


@pytest.mark.parametrize("cl", [True, False])
def test_global_avgpool_grad_and_layout(cl):
    """FusedGlobalAvgPool2d == AdaptiveAvgPool2d((1,1)) in value and gradient; dx keeps x's layout."""
    from madnn.nn import FusedGlobalAvgPool2d

    x = torch.randn(3, 5, 4, 6, dtype=torch.float64)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya, yb = FusedGlobalAvgPool2d((1, 1))(xa), torch.nn.AdaptiveAvgPool2d((1, 1))(xb)
    assert ya.shape == yb.shape == (3, 5, 1, 1)
    torch.testing.assert_close(ya, yb)
    g = torch.randn_like(yb)
    ya.backward(g)
    yb.backward(g)
    torch.testing.assert_close(xa.grad, xb.grad)
    assert xa.grad.is_contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format)


def test_mesh_axes_and_cp_extension_point():
    """Mesh: tp innermost, then cp, pp, dp; rank_of inverts coord; axis groups partition the world."""
    from madnn.runtime import AXES, Mesh

    m = Mesh(dp=2, pp=2, tp=2)
    assert m.cp == 1 and m.size == 8
    assert m.coords(5) == (1, 0, 1) and m.rank_of(1, 0, 1) == 5
    m4 = Mesh(dp=2, pp=2, tp=2, cp=2)
    for r in range(m4.size):
        c = m4.coord(r)
        assert m4.rank_of(c["dp"], c["pp"], c["tp"], c["cp"]) == r
    for axis in AXES:
        groups = m4.axis_groups(axis)
        assert sorted(r for g in groups for r in g) == list(range(16))
        assert all(len(g) == getattr(m4, axis) for g in groups)
    assert m4.axis_groups("tp")[0] == [0, 1] and m4.axis_groups("cp")[0] == [0, 2]


def test_fused_linear_cpu_fallback_and_reference_gelu_grad():
    """ops.linear on CPU is F.linear(+gelu); ops.bias_grad's eager path matches autograd's GELU backward."""
    from madnn import ops

    torch.manual_seed(0)
    x = torch.randn(3, 5, 16, dtype=torch.float64)
    w, b = torch.randn(24, 16, dtype=torch.float64), torch.randn(24, dtype=torch.float64)
    torch.testing.assert_close(ops.linear(x, w, b, gelu=True), F.gelu(F.linear(x, w, b), approximate="tanh"))
    pre = torch.randn(7, 24, dtype=torch.float64, requires_grad=True)
    dy = torch.randn(7, 24, dtype=torch.float64)
    F.gelu(pre, approximate="tanh").backward(dy)
    db, dp = ops.bias_grad(dy, pre.detach())
    torch.testing.assert_close(dp, pre.grad)
    torch.testing.assert_close(db, pre.grad.sum(0))


def test_auto_bucket_size():
    from madnn.config import auto_bucket_mb

    assert auto_bucket_mb(51e6) == pytest.approx(51e6 / 2**20 / 8)      # ResNet-50 bf16: ~6 MB buckets
    assert auto_bucket_mb(0.71e9) == 64.0                                 # GPT-2 medium: capped
    assert auto_bucket_mb(1e6) == 4.0                                     # tiny models: floor
    assert Config.from_env().bucket_mb == 0.0


def test_periodic_sync_counts_samples():
    """The auto-sync period is in SAMPLES (reference datamodule.lua:102,151): a 16-sample
    minibatch advances it by 16, a bare backward by 1; a sync fires on every crossed multiple."""
    from madnn.api import _PeriodicSync

    m = torch.nn.Linear(4, 2)
    ps = _PeriodicSync(m, period=10, local_size=100)
    calls = []
    ps.sync = lambda: calls.append(ps.counter)
    for _ in range(3):  # 16-sample minibatches: 16, 32, 48 cross 10, 30, 40
        ps.count_next(16)
        m(torch.randn(16, 4)).sum().backward()
    assert ps.counter == 48 and calls == [16, 32, 48]
    for _ in range(2):  # per-sample backward: 49, 50 -> crosses 50
        m(torch.randn(1, 4)).sum().backward()
    assert ps.counter == 50 and calls[-1] == 50 and ps.backwards == 5


def test_step_profiler_writes_a_trace(tmp_path):
    from madnn.models import MLP
    from madnn.utils.profiling import kernel_table, step_profiler

    m = MLP(8, 16, 4)
    x = torch.randn(4, 8)
    with step_profiler(str(tmp_path), wait=0, warmup=1, active=2) as prof:
        for _ in range(3):
            m(x).sum().backward()
            prof.step()
    trace = (tmp_path / "trace-rank0.json").read_text()
    assert "addmm" in trace or "linear" in trace
    assert isinstance(kernel_table(prof), str)


def test_shipped_tuning_table_covers_bench_shapes(monkeypatch):
    """The shipped per-shape table (madnn/tuning/choices_gfx950.json) holds every weight-gradient
    and GELU-Linear shape of the bench configurations, so a bench process times nothing at start
    (round 3: 76 s of first-step timing + MIOpen search, profiles/r4_first_steps_*.json)."""
    import madnn.ops as ops

    assert ops._TUNE["table"] and ops._TUNE["table"].endswith("choices_gfx950.json")
    # ResNet-50 at 2048 and 512 images: the layer1 1x1 conv3 weight gradient, the 3x3 of layer4
    for b in (2048, 512):
        assert ("conv1x1", b * 56 * 56, 256, 64) in ops._WGRAD_CHOICE
        assert ("conv3x3", b, 512, 7, 7, 512) in ops._WGRAD_CHOICE
    # GPT-2 medium at every microbatch the pipeline planner may pick (4 .. 64 sequences)
    for b in (4, 8, 16, 32, 64):
        assert ("linear", b * 1024, 4096, 1024) in ops._WGRAD_CHOICE

    def boom(*a, **k):
        raise AssertionError("a shipped shape was timed")

    monkeypatch.setattr(ops, "_time_wgrad", boom)
    called = []
    key = ("conv1x1", 2048 * 56 * 56, 256, 64)
    ops.tuned_wgrad(key, lambda: called.append("lib"), lambda: called.append("k12"),
                    k9=lambda: called.append("k9"), k12w=lambda: called.append("k12w"),
                    k12wh=lambda: called.append("k12wh"))
    assert called == [ops._WGRAD_CHOICE[key]] and ops.tuning_timings() == 0


def test_tuning_table_roundtrip(tmp_path):
    import madnn.ops as ops

    p = tmp_path / "t.json"
    ops.export_choices(str(p))
    saved = dict(ops._WGRAD_CHOICE)
    ops._WGRAD_CHOICE.clear()
    try:
        assert ops.load_tuning_table(str(p)) >= len(saved)
        assert ops._WGRAD_CHOICE == saved
    finally:
        ops._WGRAD_CHOICE.update(saved)
        ops.load_tuning_table()


def test_planner_prices_pipelines_with_the_engine_transport():
    """transport_time = the simulated makespan of the engine's own transport: with free transfers
    it is the compute-only schedule (M*chunk / (1 - bubble)); with transfers it grows, and it is
    the better of the engine's two issue plans: the one placed on a clock that includes the
    transfer time hides most of GPipe's transfers, which the lag-0 plan leaves exposed."""
    from madnn.parallel.pp import pipeline_bubble, simulate_transport, transport_time

    chunk = 3e-3
    for kind, V in (("gpipe", 1), ("1f1b", 1), ("interleaved", 2)):
        free = transport_time(kind, 4, 16, V, chunk / V, 0.0)
        ideal = 16 * chunk / (1 - pipeline_bubble(kind, 4, 16, V))
        assert free == pytest.approx(ideal, rel=1e-9)
        assert transport_time(kind, 4, 16, V, chunk / V, 0.25 * chunk / V) > free
    # a transfer of a quarter of a microbatch forward (chunk = forward + backward = 3 forwards)
    exp = {k: transport_time(k, 4, 16, 1, chunk, chunk / 12) / transport_time(k, 4, 16, 1, chunk, 0.0)
           for k in ("gpipe", "1f1b")}
    lag0 = {k: simulate_transport(k, 4, 16, 1, "split", None, t_p2p=0.25)["makespan"]
            / simulate_transport(k, 4, 16, 1, "split", None)["makespan"] for k in ("gpipe", "1f1b")}
    assert 1.0 < exp["1f1b"] <= lag0["1f1b"] and 1.0 < exp["gpipe"] < lag0["gpipe"]


def test_chain_calibration_rescales_activation_memory_at_a_batch_that_fits(monkeypatch):
    """When the estimated activations of the timing batch would not fit half of HBM, the chain
    forward runs at the largest batch that does: its measured saved bytes rescale every layer's
    act_bytes (the estimate over-counts most exactly when it is large), and the timing ratio,
    which a smaller batch would distort, is left alone."""
    import madnn.planner as planner
    from madnn.planner.cost import LayerCost
    from madnn.planner.hw import load

    hw = load()
    costs = [LayerCost(name=f"l{i}", params=1000, shared_params=0, flops=1.0, act_bytes=1e9, out_bytes=1.0,
                       fwd_s=1e-3, bwd_s=2e-3, measured=True) for i in range(4)]
    seen = {}

    def fake_chain(spine, example_input, costs_, *, batch, dtype=None, saved=None, **kw):
        seen["batch"] = batch
        saved["bytes"] = 0.4 * 4e9 * batch       # 40 % of the estimate is really kept
        return 1.0

    monkeypatch.setattr(planner, "measure_chain", fake_chain)
    cal = planner._calibrate_chain(None, None, costs, 256, torch.bfloat16, Config(), hw)
    budget = 0.75 * hw.hbm_gb * 1e9 - 4 * 1000 * 6
    cb = 256
    while 4e9 * cb > budget:
        cb //= 2
    assert seen["batch"] == cb < 256 and cal["chain_batch"] == cb
    assert "ratio" not in cal and all(c.fwd_s == 1e-3 for c in costs)
    assert cal["act_ratio"] == pytest.approx(0.4) and all(c.act_bytes == pytest.approx(0.4e9) for c in costs)
    # a batch that fits: measured there, and the timing ratio applies
    for c in costs:
        c.act_bytes = 1e9
    layers = sum(c.call_s(8) for c in costs)
    cal = planner._calibrate_chain(None, None, costs, 8, torch.bfloat16, Config(), hw)
    assert seen["batch"] == 8 and cal["ratio"] == pytest.approx(1.0 / layers)


def test_auto_sync_period_is_the_smallest_k_within_budget():
    from madnn.parallel.dp import auto_sync_period

    assert auto_sync_period(10.0, 0.4, 0.05) == 1          # 0.4 <= 0.05 * 1 * 10
    assert auto_sync_period(10.0, 0.6, 0.05) == 2
    assert auto_sync_period(10.0, 5.0, 0.05) == 10
    assert auto_sync_period(1.0, 1e9, 0.05) == 10000       # clamped
    for step, sync in [(3.0, 0.7), (1.0, 2.5), (0.2, 0.011)]:
        k = auto_sync_period(step, sync, 0.05)
        assert sync <= 0.05 * k * step * (1 + 1e-9) and (k == 1 or sync > 0.05 * (k - 1) * step)


def test_sampler_track_sizes_dict_and_rejects_unsized_batches():
    import pytest as _pt

    from madnn.data import DistributedSampler

    s = DistributedSampler(10, rank=0, world=1, shuffle=False)
    batches = [{"input_ids": torch.zeros(3, 5), "labels": torch.zeros(3)}, (torch.zeros(2, 4), torch.zeros(2))]
    assert len(list(s.track(batches))) == 2 and s.consumed == 5
    with _pt.raises(TypeError):
        list(s.track([object()]))
    assert len(list(s.track([object()], batch_size=4))) == 1 and s.consumed == 9


def test_planned_zero_lag_is_kept():
    import types

    from madnn.parallel.pp import _DEFAULT_LAG, _planned_lag

    assert _planned_lag(types.SimpleNamespace(p2p_lag=0.0)) == 0.0
    assert _planned_lag(types.SimpleNamespace(p2p_lag=0.27)) == 0.27
    assert _planned_lag(types.SimpleNamespace()) == _DEFAULT_LAG


def test_gelu_mlp_autograd_node_matches_eager():
    """The fused MLP node (c_fc + GELU + c_proj + residual as one autograd Function) against
    eager autograd; on CPU it runs the same Function through its unfused implementations."""
    from madnn.ops import _GeluMLPFn

    torch.manual_seed(0)
    x = torch.randn(3, 5, 16, dtype=torch.float64, requires_grad=True)
    w1 = torch.randn(64, 16, dtype=torch.float64, requires_grad=True)
    b1 = torch.randn(64, dtype=torch.float64, requires_grad=True)
    w2 = torch.randn(16, 64, dtype=torch.float64, requires_grad=True)
    b2 = torch.randn(16, dtype=torch.float64, requires_grad=True)
    r = torch.randn(3, 5, 16, dtype=torch.float64, requires_grad=True)
    y = _GeluMLPFn.apply(x, w1, b1, w2, b2, r)
    gy = torch.randn_like(y)
    got = torch.autograd.grad(y, (x, w1, b1, w2, b2, r), gy)
    ref_y = torch.nn.functional.linear(torch.nn.functional.gelu(torch.nn.functional.linear(x, w1, b1),
                                                                approximate="tanh"), w2, b2) + r
    ref = torch.autograd.grad(ref_y, (x, w1, b1, w2, b2, r), gy)
    torch.testing.assert_close(y, ref_y)
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b)


def test_position_embedding_models_refuse_long_sequences():
    """GPT-2 / BERT refuse a sequence longer than their position table on the host (on the GPU the
    out-of-range gather would fault the device instead of raising)."""
    import pytest
    from madnn.models.bert import BertForPreTraining, bert_config
    from madnn.models.gpt2 import GPT2, gpt2_config

    g = GPT2(gpt2_config("gpt2-tiny"))
    with pytest.raises(ValueError, match="n_positions"):
        g(torch.zeros(1, 129, dtype=torch.long))
    b = BertForPreTraining(bert_config("bert-tiny"))
    with pytest.raises(ValueError, match="max_position"):
        b(torch.zeros(1, 129, dtype=torch.long))


def test_rope_qkv_autograd_matches_rotary_embedding():
    """ops.rope_qkv (on a view of the packed projection, eager path on CPU) equals the
    RotaryEmbedding rotation of q and k, leaves v alone, and its backward is the transpose rotation:
    gradients match autograd through the reference."""
    from madnn import ops
    from madnn.models.common import RotaryEmbedding

    torch.manual_seed(0)
    B, S, H, HKV, D = 2, 12, 4, 2, 32
    rope = RotaryEmbedding(D, 10000.0, 64)
    x = torch.randn(B, S, 16, requires_grad=True)
    w = torch.randn((H + 2 * HKV) * D, 16)
    qkv = (x @ w.t()).view(B, S, H + 2 * HKV, D)
    out = ops.rope_qkv(qkv, rope.cos, rope.sin, H + HKV)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    xr = x.detach().clone().requires_grad_(True)
    q, k, v = (xr @ w.t()).view(B, S, H + 2 * HKV, D).split([H, HKV, HKV], dim=2)
    qr, kr = rope(q, k, seq_dim=1)
    ref = torch.cat([qr, kr, v], dim=2)
    torch.testing.assert_close(out.detach(), ref.detach(), atol=1e-5, rtol=1e-5)
    (ref * g).sum().backward()
    torch.testing.assert_close(x.grad, xr.grad, atol=1e-4, rtol=1e-4)


def test_swiglu_eager_path():
    from madnn import ops

    gu = torch.randn(3, 5, 32)
    g, u = gu.chunk(2, -1)
    torch.testing.assert_close(ops.swiglu(gu), torch.nn.functional.silu(g) * u)


def test_fused_conv2d_stride2_3x3_routes_to_library_on_cpu_and_matches_conv2d():
    """FusedConv2d's stride-2 3x3 (K13 SD = 2 on the GPU for small maps) is nn.Conv2d on CPU tensors:
    same output and gradients, and the K13 predicates refuse CPU inputs."""
    from madnn import ops
    from madnn.nn.conv import FusedConv2d

    torch.manual_seed(0)
    conv = FusedConv2d(64, 64, 3, stride=2, padding=1, bias=False)
    ref = torch.nn.Conv2d(64, 64, 3, stride=2, padding=1, bias=False)
    ref.load_state_dict(conv.state_dict())
    x = torch.randn(2, 64, 14, 14, requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)
    assert not conv._k13s2(x) and not ops.conv3x3_s2_supported(x, conv.weight)
    y, part = conv(x, stats=True)
    assert part is None
    yr = ref(xr)
    torch.testing.assert_close(y, yr)
    y.sum().backward()
    yr.sum().backward()
    torch.testing.assert_close(x.grad, xr.grad)
    assert "K13" in conv.extra_repr()


def test_linear_tee_sums_the_residual_gradient_in_the_data_gradient():
    """ops._LinearTeeFn: (x W^T + b, x) with dx = dy W + d(residual) from one addmm, dW, db as eager."""
    from madnn import ops

    torch.manual_seed(0)
    x = torch.randn(3, 5, 16, requires_grad=True)
    w = torch.randn(24, 16, requires_grad=True)
    b = torch.randn(24, requires_grad=True)
    y, xr = ops._LinearTeeFn.apply(x, w, b)
    gy, gr = torch.randn_like(y), torch.randn_like(xr)
    (y * gy).sum().add((xr * gr).sum()).backward()
    xe, we, be = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    ye = torch.nn.functional.linear(xe, we, be)
    (ye * gy).sum().add((xe * gr).sum()).backward()
    torch.testing.assert_close(y, ye)
    torch.testing.assert_close(xr, x)
    for a, e in ((x.grad, xe.grad), (w.grad, we.grad), (b.grad, be.grad)):
        torch.testing.assert_close(a, e, atol=1e-5, rtol=1e-5)
    # the residual output unused: dx is the projection's data gradient alone
    x.grad = None
    y, _ = ops._LinearTeeFn.apply(x, w, b)
    (y * gy).sum().backward()
    torch.testing.assert_close(x.grad, gy.reshape(-1, 24).mm(w.detach()).view_as(x), atol=1e-5, rtol=1e-5)


def test_scaled_loss_passes_the_scale_into_scale_aware_losses():
    """ops.scaled_loss: a loss function that takes ``scale`` receives it (madnn's model losses fold
    a microbatch's 1 / M into the fused cross entropy); any other is multiplied afterwards."""
    from madnn import ops

    seen = []

    def aware(out, t, scale=1.0):
        seen.append(scale)
        return (out - t).square().mean() * scale

    def plain(out, t):
        return (out - t).square().mean()

    out, t = torch.randn(4, 3), torch.randn(4, 3)
    ref = (out - t).square().mean() * 0.25
    torch.testing.assert_close(ops.scaled_loss(aware, out, t, 0.25), ref)
    torch.testing.assert_close(ops.scaled_loss(plain, out, t, 0.25), ref)
    torch.testing.assert_close(ops.scaled_loss(plain, out, t, 1.0), (out - t).square().mean())
    assert seen == [0.25]
    # the zoo's losses take it (CPU reference path)
    from madnn.models.gpt2 import GPT2, gpt2_config

    torch.manual_seed(0)
    m = GPT2(gpt2_config("gpt2-tiny"))
    ids = torch.randint(0, 512, (2, 16))
    logits = m(ids)
    torch.testing.assert_close(ops.scaled_loss(m.loss_fn, logits, ids, 0.5), 0.5 * m.loss_fn(logits, ids))


def test_layer_fit_never_prices_a_component_at_zero_per_sample():
    """Two-point layer fit (planner.cost._fit_measurements): a forward or backward whose time did not
    grow from the quarter batch to the full batch keeps the full batch's per-sample rate (the GPU
    tier's planner test requires fwd_s, bwd_s > 0 for every layer)."""
    from madnn.planner.cost import _fit_measurements

    # (n, fwd ms, bwd ms): forward grows 4x, backward flat (0.30 ms at 64 and 0.31 ms at 16)
    fit = _fit_measurements(["a"], [[(64, 4.0, 0.30), (16, 1.0, 0.31)]])
    f, b, fixed = fit["a"]
    assert f > 0 and b > 0 and fixed >= 0
    assert abs(b - 0.30 / 64 / 1e3) < 1e-12          # the large batch's per-sample rate
    # both grow: the ordinary fixed + slope fit through the two points
    f, b, fixed = _fit_measurements(["a"], [[(64, 4.2, 8.2), (16, 1.2, 2.2)]])["a"]
    assert abs(f - 3.0 / 48 / 1e3) < 1e-12 and abs(b - 6.0 / 48 / 1e3) < 1e-12
    assert abs(fixed - (12.4 - 64 * 9.0 / 48) / 1e3) < 1e-12


def test_k12w16_asm_mfma_accumulators_are_never_copied_in_flight(tmp_path):
    """K12W16 (gemm.hip gemm4h_kernel) issues its MFMAs as asm statements, so hipcc does not know their
    AGPR results land several cycles later: the built ISA must not copy, spill or read an accumulator
    (v_accvgpr_read / write / mov, scratch traffic) between the first MFMA and the drain (s_nop 7 run)
    after the last one (checked on the gfx950 code object, no GPU needed)."""
    import shutil
    import subprocess

    so = ops.kernels_path()
    if not so.exists():
        pytest.skip("kernel library not built")
    tool = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    local = tmp_path / so.name
    shutil.copy(so, local)        # --offloading extracts next to its input
    subprocess.run([tool, "--offloading", str(local)], capture_output=True, text=True, check=True)
    body = None
    for obj in sorted(tmp_path.glob(so.name + ".*gfx950")):
        dis = subprocess.run([tool, "-d", "--mcpu=gfx950", str(obj)], capture_output=True, text=True).stdout
        start = dis.find("gemm4h_kernel")
        while start >= 0 and not dis[start:dis.find("\n", start)].endswith(">:"):
            start = dis.find("gemm4h_kernel", start + 1)
        if start >= 0:
            body = dis[start:dis.find("s_endpgm", start)]
            break
    assert body is not None, "gemm4h_kernel not in the gfx950 code object"
    ins = [ln.split("//")[0].strip() for ln in body.splitlines()[1:] if ln.strip()]
    mfma = [i for i, s in enumerate(ins) if s.startswith("v_mfma_f32_16x16x32_bf16")]
    assert len(mfma) >= 128
    drain = next(i for i in range(mfma[-1], len(ins)) if ins[i].startswith("s_nop 7"))
    bad = [s for s in ins[mfma[0]:drain]
           if s.startswith(("v_accvgpr_read", "v_accvgpr_write", "v_accvgpr_mov", "scratch_"))]
    assert not bad, bad[:5]
