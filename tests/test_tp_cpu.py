"""T1: tensor (model) parallel layers on CPU/gloo vs dense single-device layers.

Covers the reference's MP layer stack from its README (1024 -> 2048 tanh -> 10)
with the corrected semantics (SURVEY A-9..A-12): forward AND backward must match
a dense nn.Linear model for W = 2 and 4.
"""
import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from dist_utils import run_dist

pytestmark = pytest.mark.slow


def _w_row_col(rank, world):
    from madnn.nn import ColumnParallelLinear, RowParallelLinear

    torch.manual_seed(0)
    dense = nn.Linear(16, 12)
    x = torch.randn(5, 16, requires_grad=True)
    row = RowParallelLinear(16, 12)
    row.load_full(dense.weight.detach(), dense.bias.detach())
    xr = x.detach().clone().requires_grad_(True)
    y = row(xr)
    yd = dense(x)
    torch.testing.assert_close(y, yd, atol=1e-5, rtol=1e-5)
    g = torch.randn_like(yd)
    y.backward(g)
    yd.backward(g)
    torch.testing.assert_close(xr.grad, x.grad, atol=1e-5, rtol=1e-5)
    k = 16 // world
    torch.testing.assert_close(row.weight.grad, dense.weight.grad[:, rank * k:(rank + 1) * k], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(row.bias.grad, dense.bias.grad)

    col = ColumnParallelLinear(16, 12, gather_output=True)
    col.load_full(dense.weight.detach(), dense.bias.detach())
    x2 = x.detach().clone().requires_grad_(True)
    dense.zero_grad()
    x.grad = None
    y2 = col(x2)
    yd2 = dense(x)
    torch.testing.assert_close(y2, yd2, atol=1e-5, rtol=1e-5)
    y2.backward(g)
    yd2.backward(g)
    torch.testing.assert_close(x2.grad, x.grad, atol=1e-5, rtol=1e-5)
    k = 12 // world
    torch.testing.assert_close(col.weight.grad, dense.weight.grad[rank * k:(rank + 1) * k], atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("world", [2, 4])
def test_row_and_column_parallel(world):
    run_dist(_w_row_col, world)


def _w_megatron_mlp(rank, world):
    from madnn.nn import ColumnParallelLinear, RowParallelLinear

    torch.manual_seed(1)
    fc1, fc2 = nn.Linear(8, 32), nn.Linear(32, 8)
    c = ColumnParallelLinear(8, 32, gather_output=False)
    r = RowParallelLinear(32, 8, input_is_parallel=True)
    c.load_full(fc1.weight.detach(), fc1.bias.detach())
    r.load_full(fc2.weight.detach(), fc2.bias.detach())
    x = torch.randn(3, 8)
    xa = x.clone().requires_grad_(True)
    xb = x.clone().requires_grad_(True)
    ya = r(F.gelu(c(xa)))
    yb = fc2(F.gelu(fc1(xb)))
    torch.testing.assert_close(ya, yb, atol=1e-5, rtol=1e-5)
    ya.sum().backward()
    yb.sum().backward()
    torch.testing.assert_close(xa.grad, xb.grad, atol=1e-5, rtol=1e-5)


def test_megatron_mlp_ws2():
    run_dist(_w_megatron_mlp, 2)


def _w_readme_stack(rank, world):
    """README.md:97-101: MPInitialReshape(1024) -> MPInitialLinear(1024,2048) -> MPTanh -> MPBaseLinear(2048,10)."""
    import madnn.nn as mnn

    torch.manual_seed(2)
    d1, d2 = nn.Linear(1024, 2048), nn.Linear(2048, 10)
    dense = nn.Sequential(nn.Flatten(), d1, nn.Tanh(), d2)
    mp = nn.Sequential(mnn.MPInitialReshape(1024), mnn.MPInitialLinear(1024, 2048), mnn.MPTanh(),
                       mnn.MPBaseLinear(2048, 10))
    mp[1].load_full(d1.weight.detach(), d1.bias.detach())
    mp[3].load_full(d2.weight.detach(), d2.bias.detach())
    x = torch.randn(4, 32, 32)
    y = torch.randint(0, 10, (4,))
    o1 = torch.optim.SGD(dense.parameters(), lr=0.1)
    o2 = torch.optim.SGD(mp.parameters(), lr=0.1)
    for _ in range(3):
        la = F.cross_entropy(mp(x), y)
        lb = F.cross_entropy(dense(x), y)
        torch.testing.assert_close(la, lb, atol=1e-5, rtol=1e-5)
        la.backward()
        lb.backward()
        o1.step(), o2.step(), o1.zero_grad(), o2.zero_grad()
    k = 1024 // world
    torch.testing.assert_close(mp[1].weight.detach(), d1.weight.detach()[:, rank * k:(rank + 1) * k], atol=1e-5,
                               rtol=1e-5)


@pytest.mark.parametrize("world", [2, 4])
def test_reference_readme_mp_stack(world):
    run_dist(_w_readme_stack, world)


def _w_strategy_tp(rank, world):
    import madnn
    from madnn.models import MLP
    from madnn.optim import FusedSGD

    torch.manual_seed(3)
    m = MLP(64, 128, 10)
    ref = MLP(64, 128, 10)
    ref.load_state_dict(m.state_dict())
    opt = FusedSGD(m.parameters(), lr=0.1)
    m, opt = madnn.distribute(m, opt, strategy="tp", tp_min_params=1000)
    from madnn.nn import ColumnParallelLinear, RowParallelLinear

    # Megatron pairing: fc1 column-parallel (output stays sharded), fc2 row-parallel
    assert isinstance(m.fc1, ColumnParallelLinear) and not m.fc1.gather_output
    assert isinstance(m.fc2, RowParallelLinear) and m.fc2.input_is_parallel
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1)
    x, y = torch.randn(6, 64), torch.randint(0, 10, (6,))
    for _ in range(2):
        F.cross_entropy(m(x), y).backward()
        opt.step()
        opt.zero_grad()
        F.cross_entropy(ref(x), y).backward()
        ropt.step()
        ropt.zero_grad()
    torch.testing.assert_close(m(x), ref(x), atol=1e-5, rtol=1e-5)


def test_distribute_strategy_tp():
    run_dist(_w_strategy_tp, 2)


def _w_dp_tp(rank, world):
    """dp2 x tp2: each DP replica gets half the batch; equals one process on the full batch."""
    import madnn
    from madnn.models import MLP
    from madnn.optim import FusedSGD

    torch.manual_seed(4)
    m = MLP(64, 128, 10)
    ref = MLP(64, 128, 10)
    ref.load_state_dict(m.state_dict())
    opt = FusedSGD(m.parameters(), lr=0.1, momentum=0.9)
    eng, opt = madnn.distribute(m, opt, strategy="tp", tp_size=2, tp_min_params=1000)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(5)
    x, y = torch.randn(8, 64, generator=g), torch.randint(0, 10, (8,), generator=g)
    d = eng.groups.dp_idx
    for _ in range(3):
        F.cross_entropy(eng(x[d * 4:(d + 1) * 4]), y[d * 4:(d + 1) * 4]).backward()
        opt.step()
        F.cross_entropy(ref(x), y).backward()
        ropt.step()
        ropt.zero_grad()
    eng.eval()
    ref.eval()
    torch.testing.assert_close(eng(x), ref(x), atol=2e-5, rtol=2e-5)


def test_dp2_x_tp2():
    run_dist(_w_dp_tp, 4)


def _w_tp_gpt_clip_ckpt(rank, world, path):
    """dp2 x tp2 GPT-2 tiny: paired MLPs + row-parallel projections, global-norm clipping, and a
    checkpoint that holds FULL tensors (params and Adam state), consolidates into the plain
    model and resumes to the same trajectory (TP shards used to be saved as shards)."""
    import copy

    import madnn
    from madnn import ckpt
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.nn import ColumnParallelLinear, RowParallelLinear
    from madnn.optim import FusedAdam

    def make():
        torch.manual_seed(0)
        m = GPT2(gpt2_config("gpt2-tiny", n_layer=2))
        return m, FusedAdam(m.parameters(), lr=1e-2)

    m, opt = make()
    ref = copy.deepcopy(m)
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    eng, opt = madnn.distribute(m, opt, strategy="tp", tp_size=2, tp_min_params=4096)
    mlp = eng.module.h[0].mlp
    assert isinstance(mlp.c_fc, ColumnParallelLinear) and isinstance(mlp.c_proj, RowParallelLinear)
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 512, (4, 16), generator=g)
    d = eng.groups.dp_idx
    mine = ids[d * 2:(d + 1) * 2]

    def step(e, o, r=None, ro=None):
        e.module.loss_fn(e(mine), mine).backward()
        n = o.clip_grad_norm_(0.5)
        o.step()
        if r is not None:
            r.loss_fn(r(ids), ids).backward()
            rn = torch.nn.utils.clip_grad_norm_(r.parameters(), 0.5)
            torch.testing.assert_close(n, rn.detach(), atol=1e-5, rtol=1e-4)
            ro.step()
            ro.zero_grad()

    for _ in range(2):
        step(eng, opt, ref, ropt)
    ckpt.save(path, eng, opt, step=2)
    full = ckpt.consolidate(path)
    plain, _ = make()
    plain.load_state_dict(full, strict=True)  # full shapes, loads into the plain model
    for n_, p in ref.named_parameters():
        torch.testing.assert_close(full[n_], p.detach().float(), atol=3e-4, rtol=3e-4, msg=lambda m, n_=n_: f"{n_}: {m}")
    step(eng, opt)
    want = {n_: p.detach().clone() for n_, p in eng.module.named_parameters()}
    m2, opt2 = make()
    eng2, opt2 = madnn.distribute(m2, opt2, strategy="tp", tp_size=2, tp_min_params=4096)
    ckpt.load(path, eng2, opt2)
    step(eng2, opt2)
    for n_, p in eng2.module.named_parameters():
        torch.testing.assert_close(p.detach(), want[n_], atol=1e-6, rtol=1e-6, msg=n_)


def test_dp2_x_tp2_gpt_clip_and_checkpoint(tmp_path):
    run_dist(_w_tp_gpt_clip_ckpt, 4, str(tmp_path / "ck"))
