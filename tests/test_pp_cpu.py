"""T1: pipeline parallelism on CPU/gloo — parity with single-process training.

GPipe and 1F1B, 2 and 4 stages, DP x PP (2x2), tied embeddings across the
first/last stage (GPT-2), fx-split spines (an MLP without pipeline_layers).
"""
import copy

import pytest
import torch
import torch.nn.functional as F
from torch import nn

from dist_utils import run_dist

pytestmark = pytest.mark.slow


def _gpt_tiny(n_layer=4):
    from madnn.models.gpt2 import GPT2, gpt2_config

    torch.manual_seed(0)
    return GPT2(gpt2_config("gpt2-tiny", n_layer=n_layer))


class _Deep(nn.Module):
    """No pipeline_layers(): the fx tracer must find the spine."""

    def __init__(self):
        super().__init__()
        self.inp = nn.Linear(16, 32)
        self.h1 = nn.Linear(32, 32)
        self.h2 = nn.Linear(32, 32)
        self.h3 = nn.Linear(32, 32)
        self.out = nn.Linear(32, 5)

    def forward(self, x):
        x = torch.tanh(self.inp(x))
        x = torch.relu(self.h1(x)) + x
        x = torch.relu(self.h2(x))
        x = torch.relu(self.h3(x))
        return self.out(x)


def _w_pp(rank, world, model_kind, schedule, dp, microbatches, steps, clip=None, virtual=None):
    import madnn
    from madnn.optim import FusedAdam

    if model_kind in ("gpt", "gpt8"):
        model = _gpt_tiny(8 if model_kind == "gpt8" else 4)
        x = torch.randint(0, 512, (8, 32), generator=torch.Generator().manual_seed(1))
        y = x
        loss_fn = model.loss_fn
        example = x[:1]
    else:
        torch.manual_seed(0)
        model = _Deep()
        x = torch.randn(8, 16, generator=torch.Generator().manual_seed(1))
        y = torch.randint(0, 5, (8,), generator=torch.Generator().manual_seed(2))
        loss_fn = F.cross_entropy
        example = x[:1]
    ref = copy.deepcopy(model)
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.01)
    opt = FusedAdam(model.parameters(), lr=1e-2, weight_decay=0.01)
    pp = world // dp
    strategy = "pp" if dp == 1 else "dp_pp"
    eng, opt = madnn.distribute(model, opt, strategy=strategy, pp_stages=pp, microbatches=microbatches,
                                schedule=schedule, example_input=example, loss_fn=loss_fn, checkpointing="none",
                                virtual_stages=virtual, global_batch=x.shape[0])
    assert eng.plan.pp == pp and eng.plan.dp == dp
    if schedule == "interleaved":
        assert eng.V == (virtual or 2) and eng.schedule == "interleaved"
    # this replica's share of the global batch
    d_idx = eng.groups.dp_idx
    per = x.shape[0] // dp
    xr, yr = x[d_idx * per:(d_idx + 1) * per], y[d_idx * per:(d_idx + 1) * per]
    for step in range(steps):
        loss = eng.train_step(xr, yr)
        if clip is not None:
            n = opt.clip_grad_norm_(clip)
        opt.step()
        rl = loss_fn(ref(x), y)
        rl.backward()
        if clip is not None:
            rn = torch.nn.utils.clip_grad_norm_(ref.parameters(), clip)
            torch.testing.assert_close(n, rn.detach(), atol=1e-5, rtol=1e-4)  # GLOBAL norm on every rank
        ropt.step()
        ropt.zero_grad()
        if eng.holds_last and dp == 1:
            lt = 1e-5 if step < 3 else 2e-4      # Adam's drift over more steps (see below)
            torch.testing.assert_close(loss, rl.detach(), atol=lt, rtol=lt)
    from madnn.parallel.pp import _DEFAULT_LAG, plan_lag

    # the second issue plan sits at the transfer time the planner priced (or the default)
    assert eng._lags[0] == 0.0 and all(g == plan_lag(eng.plan.p2p_lag or _DEFAULT_LAG) for g in eng._lags[1:])
    if steps > 2 * len(eng._lags):
        # both issue plans ran (steps 1 .. 2L) and every rank kept the same one
        assert eng._tune["chosen"] is not None and eng.plan_lag == eng._lags[eng._tune["chosen"]]
        import torch.distributed as dist

        got = [None] * dist.get_world_size()
        dist.all_gather_object(got, eng.plan_lag)
        assert len(set(got)) == 1, got
    ref_params = dict(ref.named_parameters(remove_duplicate=False))
    mine = eng.state_dict()
    assert mine, "stage holds no parameters"
    # Adam (lr 1e-2) turns near-zero gradients into +-lr updates, so on the deeper model a few
    # elements whose gradient rounds differently across the microbatch split move by ~1e-4 (and
    # so on any model after more than a few steps)
    tol = 1e-3 if model_kind == "gpt8" or steps > 3 else 5e-5
    for name, p in mine.items():
        torch.testing.assert_close(p.detach(), ref_params[name].detach(), atol=tol, rtol=tol,
                                   msg=lambda m, name=name: f"{name}: {m}")


@pytest.mark.parametrize("schedule", ["1f1b", "gpipe"])
def test_pp_gpt_tiny_2stages(schedule):
    run_dist(_w_pp, 2, "gpt", schedule, 1, 4, 2)


def test_pp_gpt_tiny_4stages_1f1b():
    run_dist(_w_pp, 4, "gpt", "1f1b", 1, 4, 2)


def test_dp_pp_2x2_gpt_tiny():
    run_dist(_w_pp, 4, "gpt", "1f1b", 2, 2, 2)


def test_pp_fx_traced_mlp_2stages():
    run_dist(_w_pp, 2, "deep", "1f1b", 1, 2, 2)


@pytest.mark.parametrize("S,M,V", [(2, 4, 2), (2, 4, 3), (4, 4, 2)])
def test_pp_interleaved_parity(S, M, V):
    """Interleaved 1F1B (V chunks per rank, ring edge S-1 -> 0): same losses and weights as
    single-process training, tied wte/lm_head on rank 0 chunk 0 and rank S-1 chunk V-1."""
    run_dist(_w_pp, S, "gpt8" if S * V > 6 else "gpt", "interleaved", 1, M, 2, None, V)


@pytest.mark.parametrize("schedule,dp,M,V", [("1f1b", 1, 8, None), ("interleaved", 1, 8, 2), ("gpipe", 1, 4, None)])
def test_pp_4stages_parity_under_emulated_rccl(monkeypatch, schedule, dp, M, V):
    """Same parity check with every P2P batch executed the way a fully serialised RCCL rank runs
    it (rendezvous, complementary-batch check).  6 steps: the engine alternates its two issue
    plans (lag 0 / lagged) in steps 1-4 and keeps the faster from step 5 on."""
    monkeypatch.setenv("MADNN_EMULATE_RCCL_P2P", "1")
    monkeypatch.setenv("MADNN_EMULATE_RCCL_P2P_TIMEOUT", "60")
    run_dist(_w_pp, 4, "gpt8" if V else "gpt", schedule, dp, M, 6, None, V)


def test_pp_clip_grad_norm_is_global_and_tied_counted_once():
    """clip_grad_norm_ + step with tied weights across stages: the tied sum is
    applied once, and the clip coefficient uses the whole model's norm."""
    run_dist(_w_pp, 2, "gpt", "1f1b", 1, 4, 2, 0.05)


def test_dp_pp_interleaved_2x2():
    run_dist(_w_pp, 4, "gpt", "interleaved", 2, 2, 2, None, 2)


def _w_meta_tied(rank, world):
    """A META-device GPT-2 (weights never on the host) cut into 2 stages: each rank materialises
    its own stage, the tied wte / lm_head is found by NAME (ids change on
    materialisation), broadcast from the first owner and summed across the owners every step."""
    import torch.distributed as dist

    import madnn
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.optim import FusedAdam

    torch.manual_seed(0)
    with torch.device("meta"):
        model = GPT2(gpt2_config("gpt2-tiny", n_layer=4))
    opt = FusedAdam(model.parameters(), lr=1e-2)
    eng, opt = madnn.distribute(model, opt, strategy="pp", pp_stages=2, microbatches=2, checkpointing="none",
                                example_input=torch.zeros(1, 16, dtype=torch.long), global_batch=4)
    assert len(eng.tied) == 1, "tied wte/lm_head must be detected on BOTH end stages"
    ids = torch.randint(0, 512, (4, 16), generator=torch.Generator().manual_seed(2))

    def tied_value():
        p = eng.tied[0][0]
        v = eng.dp.space.master_view(p).detach().clone()
        other = v.clone()
        dist.broadcast(other, src=0)
        return v, other

    v, other = tied_value()
    torch.testing.assert_close(v, other, rtol=0, atol=0)
    for _ in range(2):
        eng.train_step(ids, ids)
        opt.step()
    v, other = tied_value()
    torch.testing.assert_close(v, other, rtol=0, atol=0)  # same summed gradient -> same update


def test_pp_meta_model_tied_weights_by_name():
    run_dist(_w_meta_tied, 2)


def _w_accumulate(rank, world):
    """two train_steps then one optimizer step equal one step on the concatenated
    batch (no tied parameters); with GPT-2's tied wte/lm_head a second train_step raises."""
    import madnn
    from madnn.optim import FusedSGD

    torch.manual_seed(0)
    model = _Deep()
    ref = copy.deepcopy(model)
    opt = FusedSGD(model.parameters(), lr=0.1)
    eng, opt = madnn.distribute(model, opt, strategy="pp", pp_stages=2, microbatches=2, schedule="1f1b",
                                example_input=torch.randn(1, 16), loss_fn=F.cross_entropy, checkpointing="none")
    g = torch.Generator().manual_seed(4)
    x, y = torch.randn(8, 16, generator=g), torch.randint(0, 5, (8,), generator=g)
    eng.train_step(x[:4], y[:4])
    eng.train_step(x[4:], y[4:])
    opt.step()
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    (F.cross_entropy(ref(x[:4]), y[:4]) + F.cross_entropy(ref(x[4:]), y[4:])).backward()
    ropt.step()
    ref_params = dict(ref.named_parameters())
    for name, p in eng.state_dict().items():
        torch.testing.assert_close(p.detach(), ref_params[name].detach(), atol=1e-5, rtol=1e-5)
    gm = _gpt_tiny()
    gopt = FusedSGD(gm.parameters(), lr=0.1)
    geng, gopt = madnn.distribute(gm, gopt, strategy="pp", pp_stages=2, microbatches=2, schedule="1f1b",
                                  example_input=torch.zeros(1, 16, dtype=torch.long), checkpointing="none")
    ids = torch.randint(0, 512, (4, 16), generator=g)
    geng.train_step(ids, ids)
    with pytest.raises(RuntimeError, match="tied"):
        geng.train_step(ids, ids)


def test_pp_gradient_accumulation_across_train_steps():
    run_dist(_w_accumulate, 2)


def _w_emulated_transport_catches_unpaired_batches(rank, world):
    import os

    import torch.distributed as dist

    from madnn.parallel.pp import P2PTransport

    os.environ["MADNN_EMULATE_RCCL_P2P"] = "1"
    os.environ["MADNN_EMULATE_RCCL_P2P_TIMEOUT"] = "30"
    tp = P2PTransport(None, dist.new_group([0, 1]), [0, 1], "cpu")
    peer = 1 - rank
    # complementary parts (an exchange) pass
    got = tp.exchange([(torch.full((3,), float(rank)), peer)], [((3,), torch.float32, peer)], "act")
    assert got[0].eq(float(peer)).all()
    # both ranks send first, each in a part of its own: gloo would buffer it, RCCL with a
    # rendezvous send and one operation at a time per rank would hang -- the emulation raises
    with pytest.raises(RuntimeError, match="transport deadlock"):
        tp.exchange([(torch.ones(3), peer)], [], "grad")


def test_emulated_serial_transport_detects_unpaired_batches():
    """Regression check of the CPU emulation itself (MADNN_EMULATE_RCCL_P2P)."""
    run_dist(_w_emulated_transport_catches_unpaired_batches, 2)


def _w_plan_tuning_with_shape_change(rank, world):
    """The issue plan of a step is a function of the step count alone: when the batch shape
    changes in the middle of the plan tuning (steps 1-4), the first / last stage exchange new
    shape headers while the interior stages do not, and every rank still runs the same plan
    (under the serial emulation a mismatch would raise "transport deadlock")."""
    import os

    import torch.distributed as dist

    import madnn
    from madnn.optim import FusedAdam

    os.environ["MADNN_EMULATE_RCCL_P2P"] = "1"
    os.environ["MADNN_EMULATE_RCCL_P2P_TIMEOUT"] = "60"
    model = _gpt_tiny(8)
    opt = FusedAdam(model.parameters(), lr=1e-3)
    eng, opt = madnn.distribute(model, opt, strategy="pp", pp_stages=4, microbatches=4, schedule="interleaved",
                                virtual_stages=2, example_input=torch.zeros(1, 32, dtype=torch.long),
                                loss_fn=model.loss_fn, checkpointing="none", global_batch=8)
    assert len(eng._lags) == 2
    g = torch.Generator().manual_seed(7)
    for step in range(7):
        seq = 32 if step != 2 else 16          # a new input signature at a tuning step
        ids = torch.randint(0, 512, (8, seq), generator=g)
        # interior ranks pass nothing: their signature stays "static", only the ends see the change
        eng.train_step(ids if eng.holds_first else None, ids if eng.holds_last else None)
        opt.step()
    got = [None] * dist.get_world_size()
    dist.all_gather_object(got, (eng.plan_lag, eng._tune["chosen"]))
    assert len(set(got)) == 1 and got[0][1] is not None, got


def test_plan_tuning_survives_a_shape_change_mid_tuning():
    run_dist(_w_plan_tuning_with_shape_change, 4)


def _w_pp_plain_optimizer(rank, world, dp, clip=None):
    """A plain torch optimizer through the pipeline path (as the DP path accepts one): the engine
    fills p.grad (after the cross-stage tied-embedding sum) before optimizer.step() and re-syncs its
    flat master copy after it -- parameters track single-process AdamW."""
    import madnn

    model = _gpt_tiny(4)
    x = torch.randint(0, 512, (8, 32), generator=torch.Generator().manual_seed(1))
    ref = copy.deepcopy(model)
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.01)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-2, weight_decay=0.01)
    pp = world // dp
    eng, opt = madnn.distribute(model, opt, strategy="pp" if dp == 1 else "dp_pp", pp_stages=pp, microbatches=2,
                                schedule="1f1b", example_input=x[:1], loss_fn=model.loss_fn, checkpointing="none",
                                global_batch=x.shape[0])
    assert isinstance(opt, torch.optim.AdamW) and eng.unpack_to_params
    d_idx = eng.groups.dp_idx
    per = x.shape[0] // dp
    xr = x[d_idx * per:(d_idx + 1) * per]
    for _ in range(3):
        eng.train_step(xr, xr)
        if clip:   # p.grad is final when train_step returns: clipping changes what the step applies
            torch.nn.utils.clip_grad_value_([p for p in model.parameters() if p.grad is not None], clip)
        opt.step()
        opt.zero_grad()
        model.loss_fn(ref(x), x).backward()
        if clip:
            torch.nn.utils.clip_grad_value_(ref.parameters(), clip)
        ropt.step()
        ropt.zero_grad()
    ref_params = dict(ref.named_parameters(remove_duplicate=False))
    for name, p in eng.state_dict().items():
        torch.testing.assert_close(p.detach(), ref_params[name].detach(), atol=1e-3, rtol=1e-3,
                                   msg=lambda m, name=name: f"{name}: {m}")


def test_pp_plain_torch_optimizer_with_grad_clipping():
    run_dist(_w_pp_plain_optimizer, 2, 1, 1e-3)


@pytest.mark.parametrize("world,dp", [(2, 1), (4, 2)])
def test_pp_plain_torch_optimizer(world, dp):
    run_dist(_w_pp_plain_optimizer, world, dp)
