"""Checkpoint format: save -> consolidate -> plain PyTorch; exact resume; re-placement
(a pipeline checkpoint restored into a data-parallel engine)."""
import copy
import os

import pytest
import torch
import torch.nn.functional as F

from dist_utils import run_dist

pytestmark = pytest.mark.slow


def _gpt():
    from madnn.models.gpt2 import GPT2, gpt2_config

    torch.manual_seed(0)
    return GPT2(gpt2_config("gpt2-tiny", n_layer=4))


def _data():
    x = torch.randint(0, 512, (8, 32), generator=torch.Generator().manual_seed(1))
    return x, x


def _w_dp_resume(rank, world, path):
    import madnn
    from madnn import ckpt
    from madnn.optim import FusedAdam

    x, y = _data()
    half = x.shape[0] // world
    xs, ys = x[rank * half:(rank + 1) * half], y[rank * half:(rank + 1) * half]

    def make():
        m = _gpt()
        o = FusedAdam(m.parameters(), lr=1e-2)
        return madnn.distribute(m, o, strategy="dp")

    eng, opt = make()
    for _ in range(2):
        F.cross_entropy(eng(xs).flatten(0, 1), ys.flatten()).backward()
        opt.step()
    ckpt.save(path, eng, opt, step=2)
    for _ in range(2):
        F.cross_entropy(eng(xs).flatten(0, 1), ys.flatten()).backward()
        opt.step()
    want = {n: p.detach().clone() for n, p in eng.module.named_parameters()}
    eng2, opt2 = make()
    meta = ckpt.load(path, eng2, opt2)
    assert meta["step"] == 2
    for _ in range(2):
        F.cross_entropy(eng2(xs).flatten(0, 1), ys.flatten()).backward()
        opt2.step()
    for n, p in eng2.module.named_parameters():
        torch.testing.assert_close(p.detach(), want[n], atol=1e-6, rtol=1e-6, msg=n)
    if rank == 0:  # consolidated checkpoint loads into the plain model
        plain = _gpt()
        plain.load_state_dict(ckpt.consolidate(path), strict=True)


def test_dp_save_resume_consolidate(tmp_path):
    run_dist(_w_dp_resume, 2, str(tmp_path / "ck"))


def _w_params_period_resume(rank, world, path):
    """sync="params" with a sample period (local_size 1200 -> 10 samples) and 4 samples a step:
    an uninterrupted run averages at steps 3, 5, 8; a run saved after step 4 and resumed must
    average at the same steps (the sample counter is restored, not restarted)."""
    import madnn
    from madnn import ckpt
    from madnn.optim import FusedSGD

    def make():
        m = _gpt()
        return madnn.distribute(m, FusedSGD(m.parameters(), lr=1e-2), strategy="dp", sync="params",
                                local_size=1200)

    x, y = _data()
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]

    def run(eng, opt, steps, synced):
        real = eng.average_parameters
        eng.average_parameters = lambda: (synced.append(eng._steps), real())
        for _ in range(steps):
            F.cross_entropy(eng(xs).flatten(0, 1), ys.flatten()).backward()
            opt.step()
        eng.average_parameters = real

    eng, opt = make()
    first = []
    run(eng, opt, 4, first)
    ckpt.save(path, eng, opt, step=4)
    rest = []
    run(eng, opt, 4, rest)
    assert first + rest == [3, 5, 8]
    eng2, opt2 = make()
    ckpt.load(path, eng2, opt2)
    assert eng2._samples == 16 and eng2._per_step == 4
    resumed = []
    run(eng2, opt2, 4, resumed)
    assert resumed == rest


def test_params_period_resumes_sample_counter(tmp_path):
    run_dist(_w_params_period_resume, 2, str(tmp_path / "ck"))


def _w_pp_save(rank, world, path):
    import madnn
    from madnn import ckpt
    from madnn.optim import FusedAdam

    m = _gpt()
    ref = copy.deepcopy(m)
    opt = FusedAdam(m.parameters(), lr=1e-2)
    eng, opt = madnn.distribute(m, opt, strategy="pp", pp_stages=world, microbatches=2, example_input=_data()[0][:1],
                                checkpointing="none")
    x, y = _data()
    eng.train_step(x, y)
    opt.step()
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    ref.loss_fn(ref(x), y).backward()
    ropt.step()
    ckpt.save(path, eng, opt, step=1)
    if rank == 0:
        full = ckpt.consolidate(path)
        for n, p in ref.state_dict().items():
            if n in full:
                torch.testing.assert_close(full[n], p.float(), atol=1e-4, rtol=1e-4, msg=lambda m: n + m)  # Adam step-1 ~ lr*sign(g)
        plain = _gpt()
        plain.load_state_dict(full, strict=False)


def _w_load_into_dp(rank, world, path):
    import madnn
    from madnn import ckpt
    from madnn.optim import FusedAdam

    m = _gpt()
    opt = FusedAdam(m.parameters(), lr=1e-2)
    eng, opt = madnn.distribute(m, opt, strategy="dp")
    ckpt.load(path, eng, opt)
    full = ckpt.consolidate(path)
    for n, p in eng.module.named_parameters():
        torch.testing.assert_close(p.detach(), full[n], msg=n)
    # optimizer state came along: one more step runs and stays finite
    x, y = _data()
    F.cross_entropy(eng(x).flatten(0, 1), y.flatten()).backward()
    opt.step()
    assert all(torch.isfinite(p).all() for p in eng.module.parameters())


def test_pp_checkpoint_restores_into_dp(tmp_path):
    path = str(tmp_path / "pp")
    run_dist(_w_pp_save, 2, path)
    assert os.path.exists(os.path.join(path, "model-00000.safetensors"))
    assert os.path.exists(os.path.join(path, "model-00001.safetensors"))
    run_dist(_w_load_into_dp, 2, path)


# ------------------------------------------------------------- resume-exact training state
class _DropNet(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(12, 32)
        self.drop = torch.nn.Dropout(0.3)   # consumes the CPU RNG: resume must restore it
        self.b = torch.nn.Linear(32, 5)

    def forward(self, x):
        return self.b(self.drop(torch.relu(self.a(x))))


def _w_mid_epoch(rank, world, path, phase):
    """Phase "save": one epoch + 3 steps, checkpoint mid-epoch, 5 more steps (losses kept).
    Phase "resume": a fresh replica (other init) loads the checkpoint and must reproduce those
    5 losses bitwise: weights, momentum, sampler cursor (same shard permutation, mid-epoch) and
    the dropout RNG all come back.  Phase "replan": the same checkpoint at another world size."""
    import madnn
    from madnn import ckpt
    from madnn.data import DistributedSampler
    from madnn.optim import FusedSGD

    g = torch.Generator().manual_seed(3)
    data, labels = torch.randn(64, 12, generator=g), torch.randint(0, 5, (64,), generator=g)
    torch.manual_seed(0 if phase == "save" else 99)
    model = _DropNet()
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9)
    eng, opt = madnn.distribute(model, opt, strategy="dp")
    sampler = DistributedSampler(len(data), shuffle=True, seed=7)
    torch.manual_seed(1000 + rank)

    def batches():
        while True:
            it = iter(sampler)
            while True:
                idx = [i for _, i in zip(range(4), it)]
                if len(idx) < 4:
                    break
                yield idx
            sampler.set_epoch(sampler.epoch + 1)

    def step(idx):
        loss = F.cross_entropy(eng(data[idx]), labels[idx])
        loss.backward()
        opt.step()
        return loss.detach().clone()

    mine = os.path.join(path, f"losses-{rank}.pt")
    if phase == "save":
        gen = batches()
        for _ in range(len(sampler) // 4 + 3):
            step(next(gen))
        assert sampler.epoch == 1 and sampler.cursor == 12
        ckpt.save(path, eng, opt, step=11, sampler=sampler)
        losses = torch.stack([step(next(gen)) for _ in range(5)])
        torch.save(losses, mine)
        return
    meta = ckpt.load(path, eng, opt, sampler=sampler)
    assert meta["step"] == 11
    if phase == "replan":
        # ranks 2 and 3 borrow the saved states of ranks 0 and 1 but must not share their
        # random streams (dropout masks), ADVICE r3
        import torch.distributed as dist

        states = [None] * world
        dist.all_gather_object(states, torch.get_rng_state().tolist())
        assert len({tuple(st) for st in states}) == world
    gen = batches()
    losses = torch.stack([step(next(gen)) for _ in range(5 if phase == "resume" else 2)])
    if phase == "resume":
        want = torch.load(mine, weights_only=True)
        assert torch.equal(losses, want), (losses, want)
    else:
        assert sampler.epoch == 1 and torch.isfinite(losses).all()


def test_mid_epoch_resume_is_bitwise_and_replans(tmp_path):
    path = str(tmp_path / "mid")
    run_dist(_w_mid_epoch, 2, path, "save")
    assert os.path.exists(os.path.join(path, "state-dp1-pp0-tp0.pt"))
    run_dist(_w_mid_epoch, 2, path, "resume")
    run_dist(_w_mid_epoch, 4, path, "replan")


def _w_trainer_resume(rank, world, path, phase):
    """parallelize() + Trainer (reference path): the periodic-sync counter, the trainer's
    epoch / position / permutation and the weights resume mid-epoch; finishing training from the
    checkpoint ends on bitwise the same weights as the uninterrupted run."""
    import madnn
    from madnn import ckpt

    g = torch.Generator().manual_seed(5)
    data, targets = torch.randn(41, 12, generator=g), torch.randint(0, 5, (41,), generator=g)
    torch.manual_seed(0 if phase == "save" else 42)
    model = torch.nn.Sequential(torch.nn.Linear(12, 16), torch.nn.Tanh(), torch.nn.Linear(16, 5))
    d, t, _ = madnn.parallelize(data, targets, model, sync_every=3, verbose=False)
    torch.manual_seed(7)

    def hook(tr, _batch):
        if phase == "save" and tr.global_step == 6:
            ckpt.save(path, model, tr.optimizer, step=tr.global_step, trainer=tr)

    tr = madnn.Trainer(model, torch.nn.CrossEntropyLoss(), learning_rate=0.2, learning_rate_decay=0.05,
                       max_iteration=3, batch_size=6, verbose=False, on_example=hook)
    if phase == "resume":
        ckpt.load(path, model, tr.optimizer, trainer=tr)
        # 20 samples per rank, batches of 6: step 6 is the 2nd step of epoch 2 (0-based epoch 1)
        assert tr.global_step == 6 and tr.epoch == 1 and tr.cursor == 12
        assert model._madnn_sync.counter == 20 + 12   # samples seen, the reference's sync unit
    tr.train(d, t)
    out = torch.cat([p.detach().flatten() for p in model.parameters()])
    f = os.path.join(path, f"final-{rank}.pt")
    if phase == "save":
        torch.save({"w": out, "syncs": model._madnn_sync.syncs, "counter": model._madnn_sync.counter}, f)
    else:
        want = torch.load(f, weights_only=True)
        assert torch.equal(out, want["w"])
        assert model._madnn_sync.counter == want["counter"]


def test_parallelize_trainer_resume_mid_epoch(tmp_path):
    path = str(tmp_path / "tr")
    run_dist(_w_trainer_resume, 2, path, "save")
    run_dist(_w_trainer_resume, 2, path, "resume")


def test_sampler_resume_counts_consumed_not_prefetched():
    """A DataLoader with workers pulls batches ahead of training; the saved position is what the
    loop consumed (``DistributedSampler.track``), so resume continues at the first UNtrained
    batch instead of skipping the prefetched ones."""
    from madnn.data import DistributedSampler

    data = torch.arange(64)
    ds = torch.utils.data.TensorDataset(data)
    s = DistributedSampler(64, rank=0, world=1, shuffle=True, seed=3)
    loader = torch.utils.data.DataLoader(ds, batch_size=4, sampler=s, num_workers=2, prefetch_factor=2)
    seen = []
    for i, (b,) in enumerate(s.track(loader)):
        seen += b.tolist()
        if i == 4:
            sd = s.state_dict()
            ahead = s.cursor
            break
    assert sd["cursor"] == 20 and ahead > 20          # the workers had handed out more
    r = DistributedSampler(64, rank=0, world=1, shuffle=True, seed=3)
    r.load_state_dict(sd)
    rest = list(iter(r))
    full = list(iter(DistributedSampler(64, rank=0, world=1, shuffle=True, seed=3)))
    assert seen == full[:20] and rest == full[20:]
    # the hand-loop API: advance() after each step
    a = DistributedSampler(64, rank=0, world=1, shuffle=False)
    it = iter(a)
    for _ in range(8):
        next(it)                  # 8 handed out (a prefetching loop) ...
    a.advance(4)                  # ... 4 trained
    assert a.state_dict()["cursor"] == 4


def test_resume_on_larger_tp_mesh_keeps_tp_groups_on_one_rng_stream(tmp_path, monkeypatch):
    """a rank resumed on a larger mesh borrows a saved coordinate's RNG state; the
    dp / pp coordinates are folded in (replicas draw different masks), the tp coordinate is not
    (a tensor-parallel group keeps one shared stream)."""
    import types

    from madnn import ckpt

    g = torch.Generator()
    g.manual_seed(7)
    shared = g.get_state()          # saved at dp=1 x tp=2: both tp ranks on one stream
    for tp in range(2):
        torch.save({"rng_cpu": shared.clone()}, str(tmp_path / f"state-dp0-pp0-tp{tp}.pt"))
    meta = {"mesh": {"dp": 1, "pp": 1, "tp": 2}}

    def state_at(dp, tp):
        eng = types.SimpleNamespace(groups=types.SimpleNamespace(dp_idx=dp, pp_idx=0, tp_idx=tp))
        return ckpt._load_resume_state(str(tmp_path), eng, meta)["rng_cpu"]

    # resumed at dp=2 x tp=4: every rank of one TP group shares a stream ...
    for dp in range(2):
        states = [state_at(dp, tp) for tp in range(4)]
        for s in states[1:]:
            assert torch.equal(s, states[0])
    # ... the saved replica keeps its own, the new replica gets a different one
    assert torch.equal(state_at(0, 3), shared)
    assert not torch.equal(state_at(1, 0), shared)


def _w_pp_plain_opt_resume(rank, world, path, phase):
    """Pipeline engine + plain torch AdamW: save after 2 steps, then either keep training (phase
    "save", losses kept) or resume a fresh replica from the checkpoint (phase "resume"): the next
    steps' losses must match -- weights AND the AdamW moments come back through the checkpoint."""
    import madnn
    from madnn import ckpt

    torch.manual_seed(0 if phase == "save" else 42)
    m = _gpt()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-2, weight_decay=0.01)
    eng, opt = madnn.distribute(m, opt, strategy="pp", pp_stages=world, microbatches=2,
                                example_input=_data()[0][:1], checkpointing="none")
    assert isinstance(opt, torch.optim.AdamW)
    x, y = _data()

    def step():
        loss = eng.train_step(x, y)
        opt.step()
        opt.zero_grad()
        return torch.as_tensor(float(loss) if loss is not None else 0.0)

    mine = os.path.join(path, f"plain-losses-{rank}.pt")
    if phase == "save":
        step()
        step()
        ckpt.save(path, eng, opt, step=2)
        torch.save(torch.stack([step() for _ in range(3)]), mine)
        return
    ckpt.load(path, eng, opt)
    got = torch.stack([step() for _ in range(3)])
    want = torch.load(mine, weights_only=True)
    torch.testing.assert_close(got, want, atol=1e-5, rtol=1e-5)


def test_pp_plain_optimizer_checkpoint_resume(tmp_path):
    path = str(tmp_path / "pp_plain")
    run_dist(_w_pp_plain_opt_resume, 2, path, "save")
    run_dist(_w_pp_plain_opt_resume, 2, path, "resume")
