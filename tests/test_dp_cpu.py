"""T1: data parallelism on CPU/gloo, world_size 2 (BASELINE config 1: 2-layer MLP auto-DP).

Parity criteria: ws=2 with per-rank batch b equals one process
with batch 2b; the reference's periodic parameter averaging with K=1 and plain
SGD equals gradient averaging (Appendix A-3); reference sharding semantics.
"""
import copy

import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F

from dist_utils import run_dist

pytestmark = pytest.mark.slow

B = 8


def _data(seed=0, n=4 * B):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 32, generator=g), torch.randint(10, (n,), generator=g)


def _ref_model():
    from madnn.models import MLP

    torch.manual_seed(0)
    return MLP(32, 64, 10)


def _check_same_across_ranks(t):
    ts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(ts, t.contiguous())
    for o in ts[1:]:
        torch.testing.assert_close(o, ts[0], rtol=0, atol=0)


def _w_dp_parity(rank, world, opt_kind, bucket_mb, sync):
    import madnn
    from madnn.optim import FusedAdam, FusedSGD

    model = _ref_model()
    ref = copy.deepcopy(model)
    if rank == 1:  # replicas start different: the engine must broadcast rank 0's weights
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    if opt_kind == "sgd":
        opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-3)
        ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-3)
    elif opt_kind == "adam":
        opt = FusedAdam(model.parameters(), lr=1e-2, weight_decay=1e-2)
        ropt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=1e-2)
    else:  # plain torch optimizer through the engine's unpack path
        opt = torch.optim.SGD(model.parameters(), lr=0.1)
        ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    dm, opt = madnn.distribute(model, opt, strategy="dp", bucket_mb=bucket_mb, sync=sync, sync_every=1)
    x, y = _data()
    for step in range(4):
        xs = x[step * B:(step + 1) * B]
        ys = y[step * B:(step + 1) * B]
        half = B // world
        loss = F.cross_entropy(dm(xs[rank * half:(rank + 1) * half]), ys[rank * half:(rank + 1) * half])
        loss.backward()
        opt.step()
        opt.zero_grad()
        rl = F.cross_entropy(ref(xs), ys)
        rl.backward()
        ropt.step()
        ropt.zero_grad()
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), atol=2e-5, rtol=2e-5)
        _check_same_across_ranks(p.detach())


@pytest.mark.parametrize("opt_kind", ["sgd", "adam", "torch"])
def test_dp_grad_parity_ws2(opt_kind):
    run_dist(_w_dp_parity, 2, opt_kind, 64.0, "grads")


def test_dp_many_small_buckets_ws2():
    run_dist(_w_dp_parity, 2, "sgd", 0.0005, "grads")  # ~128 fp32 elems per bucket => one bucket per tensor


def _w_params_mode(rank, world):
    """A-3: periodic parameter averaging with K=1 and vanilla SGD == gradient averaging."""
    import madnn
    from madnn.optim import FusedSGD

    x, y = _data(1)
    outs = {}
    for sync in ("grads", "params"):
        model = _ref_model()
        opt = FusedSGD(model.parameters(), lr=0.05)
        dm, opt = madnn.distribute(model, opt, strategy="dp", sync=sync, sync_every=1)
        for step in range(3):
            xs = x[step * B + rank * 4: step * B + rank * 4 + 4]
            ys = y[step * B + rank * 4: step * B + rank * 4 + 4]
            F.cross_entropy(dm(xs), ys).backward()
            opt.step()
            opt.zero_grad()
        outs[sync] = [p.detach().clone() for p in model.parameters()]
    for a, b in zip(outs["grads"], outs["params"]):
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)


def test_params_mode_equals_grads_mode_k1():
    run_dist(_w_params_mode, 2)


def _w_params_period(rank, world, mode):
    """``distribute(sync="params")`` period: None -> the reference heuristic in SAMPLES on the
    local shard (R6, datamodule.lua:68-78); "auto" -> K measured on the job, agreed by all ranks."""
    import madnn
    from madnn.data import shard
    from madnn.optim import FusedSGD
    from madnn.parallel.dp import auto_sync_period

    x, y = _data(3, n=2400)
    xs, ys = shard(x), shard(y)                       # 1200 local samples -> heuristic 10 samples
    assert len(xs) == 1200
    model = _ref_model()
    opt = FusedSGD(model.parameters(), lr=0.05)
    kw = {"sync_every": "auto", "sync_budget": 1e6 if mode == "auto_k1" else 1e-6} if mode != "none" else {}
    dm, opt = madnn.distribute(model, opt, strategy="dp", sync="params", **kw)
    synced = []
    real = dm.average_parameters

    def counting():
        synced.append(dm._steps)
        real()

    dm.average_parameters = counting
    for step in range(8):
        F.cross_entropy(dm(xs[step * 4:step * 4 + 4]), ys[step * 4:step * 4 + 4]).backward()
        opt.step()
        opt.zero_grad()
        if step + 1 in synced:
            for p in model.parameters():
                _check_same_across_ranks(p.detach())
    if mode == "none":
        assert dm.sync_samples == 10
        assert synced == [3, 5, 8]                   # 4 samples per step: crossing 10, 20, 30
        return
    cal = dm.sync_calibration
    assert cal is not None and cal["decided_at_step"] == 4
    k = torch.tensor([float(cal["K"]), cal["step_ms"], cal["sync_ms"]], dtype=torch.float64)
    _check_same_across_ranks(k)                      # every rank chose the same K from the same MAXes
    assert cal["K"] == auto_sync_period(cal["step_ms"], cal["sync_ms"], cal["budget"])
    assert synced[:4] == [1, 2, 3, 4]                # K = 1 while measuring
    if mode == "auto_k1":
        assert cal["K"] == 1 and synced == list(range(1, 9))
    else:
        assert cal["K"] == 10000 and synced == [1, 2, 3, 4]
    assert dm.sync_every == cal["K"]


@pytest.mark.parametrize("mode", ["none", "auto_k1", "auto_kmax"])
def test_distribute_params_sync_period(mode):
    run_dist(_w_params_period, 2, mode)


def _w_params_period_unequal_shards(rank, world):
    """Shards of 2499 and 2500 samples (``remainder="last"``) fall into different tiers of the
    reference heuristic (10 vs 50 samples), and the ranks train different batch sizes: the period
    and the per-step sample count are agreed, so both ranks average at the same steps."""
    import madnn
    from madnn.data import shard
    from madnn.optim import FusedSGD

    x, y = _data(5, n=4999)
    xs, ys = shard(x, remainder="last"), shard(y, remainder="last")
    assert len(xs) == (2499 if rank == 0 else 2500)
    model = _ref_model()
    opt = FusedSGD(model.parameters(), lr=0.05)
    dm, opt = madnn.distribute(model, opt, strategy="dp", sync="params")
    assert dm.sync_samples == 10                      # the smaller shard's tier, on both ranks
    synced = []
    real = dm.average_parameters

    def counting():
        synced.append(dm._steps)
        real()

    dm.average_parameters = counting
    b = 3 if rank == 0 else 4                          # 3 samples a step are agreed
    for step in range(10):
        F.cross_entropy(dm(xs[step * b:step * b + b]), ys[step * b:step * b + b]).backward()
        opt.step()
        opt.zero_grad()
    assert synced == [4, 7, 10], synced               # crossing 10, 20, 30 at 3 samples a step
    _check_same_across_ranks(torch.tensor(synced))
    for p in model.parameters():
        _check_same_across_ranks(p.detach())


def test_params_period_agreed_with_unequal_shards():
    run_dist(_w_params_period_unequal_shards, 2)


def _w_no_sync(rank, world):
    import madnn
    from madnn.optim import FusedSGD

    model = _ref_model()
    ref = copy.deepcopy(model)
    opt = FusedSGD(model.parameters(), lr=0.1)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    dm, opt = madnn.distribute(model, opt, strategy="dp")
    x, y = _data(2)
    # two micro-batches per rank accumulated locally, reduced once
    with dm.no_sync():
        F.cross_entropy(dm(x[rank * 4:rank * 4 + 4]), y[rank * 4:rank * 4 + 4]).backward()
    F.cross_entropy(dm(x[8 + rank * 4:8 + rank * 4 + 4]), y[8 + rank * 4:8 + rank * 4 + 4]).backward()
    opt.step()
    l1 = F.cross_entropy(ref(x[0:8]), y[0:8])
    l2 = F.cross_entropy(ref(x[8:16]), y[8:16])
    ((l1 + l2)).backward()
    ropt.step()
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), atol=2e-5, rtol=2e-5)


def test_no_sync_accumulation():
    run_dist(_w_no_sync, 2)


def _w_unused(rank, world):
    import madnn
    from madnn.optim import FusedSGD

    class Two(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.a = torch.nn.Linear(4, 4)
            self.b = torch.nn.Linear(4, 4)  # never used

        def forward(self, x):
            return self.a(x)

    torch.manual_seed(0)
    m = Two()
    opt = FusedSGD(m.parameters(), lr=0.1)
    dm, opt = madnn.distribute(m, opt, strategy="dp", bucket_mb=0.00001)
    before = m.b.weight.detach().clone()
    dm(torch.randn(3, 4)).sum().backward()
    opt.step()
    torch.testing.assert_close(m.b.weight.detach(), before)


def test_unused_parameters():
    run_dist(_w_unused, 2)


# ------------------------------------------------------------- reference API
def _w_synchronize_model(rank, world):
    import madnn

    torch.manual_seed(rank)
    m = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Tanh(), torch.nn.Linear(7, 3))
    for p in m.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    mine = [p.detach().clone() for p in m.parameters()]
    allp = [[torch.empty_like(t) for _ in range(world)] for t in mine]
    for t, lst in zip(mine, allp):
        dist.all_gather(lst, t)
    madnn.synchronize_model(m)
    for p, lst in zip(m.parameters(), allp):
        torch.testing.assert_close(p.detach(), sum(lst) / world, atol=1e-6, rtol=1e-6)
        torch.testing.assert_close(p.grad, torch.full_like(p, 1.5))


def test_synchronize_model_averages_params_and_grads():
    run_dist(_w_synchronize_model, 2)


def _w_parallelize(rank, world, sync_every):
    import madnn
    from madnn.models import MLP

    torch.manual_seed(10 + rank)  # different init per rank: parallelize must broadcast
    g = torch.Generator().manual_seed(0)
    n = 203
    w_true = torch.randn(16, 3, generator=g)
    data = torch.randn(n, 16, generator=g)
    targets = (data @ w_true).argmax(1)
    model = MLP(16, 32, 3)
    d, t, size = madnn.parallelize(data, targets, model, sync_every=sync_every, verbose=False)
    assert size == n // world == len(d) == len(t)
    torch.testing.assert_close(d, data[rank * size:(rank + 1) * size])  # contiguous stripe, remainder dropped
    if sync_every is None:
        assert model._madnn_sync.period == 1  # heuristic: local size < 1000
    lrs, iters = [], []

    def hook(tr, it, err):
        lrs.append(tr.optimizer.param_groups[0]["lr"])
        iters.append(it)

    trainer = madnn.Trainer(model, torch.nn.CrossEntropyLoss(), learning_rate=0.5, learning_rate_decay=0.1,
                            max_iteration=6, batch_size=16, verbose=False, on_iteration=hook)
    from madnn.optim import FusedSGD

    assert isinstance(trainer.optimizer, FusedSGD)  # the reference's fused accUpdateGradParameters
    hist = trainer.train(d, t)
    assert hist[-1] < hist[0]
    assert trainer.optimizer.space is not None and len(trainer.optimizer.space.buckets) >= 1
    # reference schedule (datamodule.lua:176-177): epoch 1 at lr, epoch k >= 2 at lr / (1 + k * decay)
    assert lrs == pytest.approx([0.5] + [0.5 / (1 + k * 0.1) for k in range(2, 7)])
    # hookIteration receives the 1-based iteration (datamodule.lua:169-170)
    assert iters == [1, 2, 3, 4, 5, 6]
    # maxIteration <= 0: no limit (datamodule.lua:178); the hook ends training with StopIteration
    seen = []

    def stop_at_3(tr, it, err):
        seen.append(it)
        if it == 3:
            raise StopIteration

    t2 = madnn.Trainer(model, torch.nn.CrossEntropyLoss(), learning_rate=0.05, max_iteration=0, batch_size=16,
                       verbose=False, on_iteration=stop_at_3)
    assert len(t2.train(d, t)) == 3 and seen == [1, 2, 3] and t2.epoch == 3
    if sync_every == -1:
        madnn.synchronize_model(model)
    for p in model.parameters():
        _check_same_across_ranks(p.detach())


@pytest.mark.parametrize("sync_every", [None, 3, -1])
def test_parallelize_trainer(sync_every):
    run_dist(_w_parallelize, 2, sync_every)


def _w_ws4(rank, world):
    _w_dp_parity(rank, world, "sgd", 64.0, "grads")


def test_dp_parity_ws4():
    run_dist(_w_ws4, 4)


def _metrics_worker(rank, world, path):
    import json

    import madnn
    from madnn.models import MLP
    from madnn.optim import FusedSGD
    from madnn.utils.metrics import StepMeter

    torch.manual_seed(0)
    model = MLP(16, 32, 4)
    opt = FusedSGD(model.parameters(), lr=0.1)
    eng, opt = madnn.distribute(model, opt, strategy="dp")
    meter = StepMeter(eng, samples_per_step=8 * world, path=path if rank == 0 else None)
    x, y = torch.randn(8, 16), torch.randint(0, 4, (8,))
    for _ in range(3):
        meter.start()
        loss = torch.nn.functional.cross_entropy(eng(x), y)
        loss.backward()
        opt.step()
        m = meter.stop(loss)
    meter.close()
    assert m["allreduce_bytes"] > 0 and m["samples_per_s"] > 0 and m["step"] == 3
    if rank == 0:
        rows = [json.loads(l) for l in open(path)]
        assert len(rows) == 3 and all("loss" in r and "step_ms" in r for r in rows)


def test_step_metrics_jsonl(tmp_path):
    run_dist(_metrics_worker, 2, str(tmp_path / "metrics.jsonl"))


# ------------------------------------------------------- bucket layout / grad sinks
class _Crossed(torch.nn.Module):
    """Registration order differs from backward order: ``late`` is registered first but is used
    LAST in forward (so its gradient arrives first), ``early`` the other way round."""

    def __init__(self):
        super().__init__()
        self.late = torch.nn.Linear(16, 4)
        self.mid = torch.nn.Linear(16, 16)
        self.early = torch.nn.Linear(8, 16)

    def forward(self, x):
        return self.late(torch.relu(self.mid(torch.relu(self.early(x)))))


def _w_relayout(rank, world):
    import madnn
    from madnn.optim import FusedSGD

    torch.manual_seed(0)
    m = _Crossed()
    ref = copy.deepcopy(m)
    opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.9)
    # tiny buckets: one or two parameters each, so the order matters
    dm, opt = madnn.distribute(m, opt, strategy="dp", bucket_mb=300 * 4 / 2**20)
    nb = len(dm.space.buckets)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(1)
    for step in range(3):
        x, y = torch.randn(4 * world, 8, generator=g), torch.randint(0, 4, (4 * world,), generator=g)
        F.cross_entropy(dm(x[4 * rank:4 * rank + 4]), y[4 * rank:4 * rank + 4]).backward()
        opt.step()
        F.cross_entropy(ref(x), y).backward()
        ropt.step()
        ropt.zero_grad()
        if step == 0:
            assert dm.rebuilt, "buckets should follow the observed gradient order after step 1"
            assert dm.space.layout_is_contiguous([id(p) for p in (m.late.bias, m.late.weight, m.mid.bias,
                                                                  m.mid.weight, m.early.bias, m.early.weight)])
    assert len(dm.space.buckets) == nb
    for p, q in zip(m.parameters(), ref.parameters()):  # values and momentum migrated exactly
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_buckets_relaid_in_observed_order():
    run_dist(_w_relayout, 2)


class _RankOrdered(torch.nn.Module):
    """Rank 0 runs a then b, rank 1 b then a: the two replicas OBSERVE opposite gradient orders."""

    def __init__(self, rank):
        super().__init__()
        self.rank = rank
        self.a = torch.nn.Linear(16, 16)
        self.b = torch.nn.Linear(16, 16)
        self.head = torch.nn.Linear(16, 4)

    def forward(self, x):
        h = self.b(torch.tanh(self.a(x))) if self.rank == 0 else self.a(torch.tanh(self.b(x)))
        return self.head(h)


def _w_relayout_disagree(rank, world):
    """replicas re-lay their buckets by ONE agreed order (the source rank's), so the
    bucket all-reduces keep summing matching slices and the weights stay identical."""
    import madnn
    from madnn.optim import FusedSGD

    torch.manual_seed(0)
    m = _RankOrdered(rank)
    opt = FusedSGD(m.parameters(), lr=0.1)
    dm, opt = madnn.distribute(m, opt, strategy="dp", bucket_mb=300 * 4 / 2**20)
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        x, y = torch.randn(4, 16, generator=g), torch.randint(0, 4, (4,), generator=g)
        F.cross_entropy(dm(x), y).backward()
        opt.step()
    names = {id(p): n for n, p in m.named_parameters()}
    layout = [[names[id(p)] for p in bk.params] for bk in dm.space.buckets]
    objs = [None] * world
    dist.all_gather_object(objs, layout)
    assert objs[0] == objs[1], objs
    for p in m.parameters():
        _check_same_across_ranks(p.detach())


def test_relayout_agrees_across_ranks():
    run_dist(_w_relayout_disagree, 2)


def test_grad_sink_writes_in_place_cpu():
    """ops.linear's backward writes the weight gradient straight into the bucket slot and
    autograd adopts that view as p.grad (no copy); the reducer then skips it when packing."""
    from madnn import ops
    from madnn.parallel.flat import FlatParamSpace

    torch.manual_seed(0)
    lin = torch.nn.Linear(16, 8)
    ref = copy.deepcopy(lin)
    space = FlatParamSpace([list(lin.parameters())], dtype_of=lambda p: torch.float32, bucket_cap_mb=1.0)
    assert space.enable_grad_sinks() == 2
    x = torch.randn(5, 16)
    ops.linear(x, lin.weight, lin.bias, force_fn=True).square().sum().backward()
    ref(x).square().sum().backward()
    bk, off, _ = space.param_info[id(lin.weight)]
    assert lin.weight.grad.data_ptr() == bk.grad.data_ptr() + off * 4, "weight grad was copied"
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad)
    ts, offs, missing = space.bucket_grads(bk)
    assert all(t is not lin.weight.grad for t in ts) and id(lin.weight) not in [id(t) for t in ts]
    assert space.packed_fraction(bk) < 0.1  # only the bias (K11 column sum) is packed
    # a second accumulation (no_sync microbatch) adds in place into the same slot
    ops.linear(x, lin.weight, lin.bias, force_fn=True).square().sum().backward()
    torch.testing.assert_close(lin.weight.grad, 2 * ref.weight.grad)


def _w_bf16_reduce(rank, world, out_dir):
    """reduce_dtype="auto" all-reduces bf16 parameters' gradient buckets in bf16. At
    8 ranks that tracks the fp32 reduction within bf16 rounding (checked against an fp32-reduce
    run of the same bf16 model and against fp32 single-process training)."""
    import madnn
    from madnn.models import MLP
    from madnn.optim import FusedSGD

    g = torch.Generator().manual_seed(9)
    x, y = torch.randn(8 * world, 32, generator=g), torch.randint(0, 10, (8 * world,), generator=g)
    finals = {}
    for rd in ("auto", "float32"):
        torch.manual_seed(0)
        m = MLP(32, 64, 10)
        opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.9)
        eng, opt = madnn.distribute(m, opt, strategy="dp", reduce_dtype=rd, cpu_dtype="bfloat16")
        assert {bk.grad_dtype for bk in eng.space.buckets} == ({torch.bfloat16} if rd == "auto" else {torch.float32})
        for _ in range(3):
            xs, ys = x[rank * 8:(rank + 1) * 8], y[rank * 8:(rank + 1) * 8]
            F.cross_entropy(eng(xs).float(), ys).backward()
            opt.step()
        finals[rd] = torch.cat([eng.space.master_view(p).flatten() for p in m.parameters()])
        eng.remove_hooks()
    torch.manual_seed(0)
    ref = MLP(32, 64, 10)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    for _ in range(3):
        F.cross_entropy(ref(x), y).backward()
        ropt.step()
        ropt.zero_grad()
    want = torch.cat([p.detach().flatten() for p in ref.parameters()])
    d_auto = (finals["auto"] - want).abs().max().item()
    d_f32 = (finals["float32"] - want).abs().max().item()
    # bf16 compute dominates the error; the bf16 reduction adds at most its own rounding on top
    assert d_auto < 3e-2 and d_f32 < 3e-2, (d_auto, d_f32)
    assert (finals["auto"] - finals["float32"]).abs().max().item() < 2e-2
    _check_same_across_ranks(finals["auto"])


def test_bf16_reduce_tracks_fp32_reduce_at_8_ranks(tmp_path):
    run_dist(_w_bf16_reduce, 8, str(tmp_path))


def _w_bf16_sync(rank, world):
    import madnn

    torch.manual_seed(0)
    base = torch.randn(257, 33)
    m = torch.nn.Linear(33, 257).to(torch.bfloat16)
    with torch.no_grad():
        m.weight.copy_((base * (1 + rank / 7.0)).to(torch.bfloat16))
        m.bias.fill_(1.0 + rank * 2 ** -9)
    want_w = sum((base * (1 + r / 7.0)).to(torch.bfloat16).float() for r in range(world)) / world
    want_b = sum(torch.tensor(1.0 + r * 2 ** -9).to(torch.bfloat16).float() for r in range(world)) / world
    madnn.synchronize_model(m, grads=False)
    # one rounding of the fp32 mean, not a bf16 running sum
    assert torch.equal(m.weight, want_w.to(torch.bfloat16))
    assert torch.equal(m.bias, want_b.to(torch.bfloat16).expand_as(m.bias))


def test_bf16_synchronize_model_sums_in_fp32():
    """averaging a bf16 model reduces the W-rank sum in fp32 (8 ranks)."""
    run_dist(_w_bf16_sync, 8)
