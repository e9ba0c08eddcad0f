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


def _gpt_tiny():
    from madnn.models.gpt2 import GPT2, gpt2_config

    torch.manual_seed(0)
    return GPT2(gpt2_config("gpt2-tiny", n_layer=4))


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


def _w_pp(rank, world, model_kind, schedule, dp, microbatches, steps):
    import madnn
    from madnn.optim import FusedAdam

    if model_kind == "gpt":
        model = _gpt_tiny()
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
                                schedule=schedule, example_input=example, loss_fn=loss_fn, checkpointing="none")
    assert eng.plan.pp == pp and eng.plan.dp == dp
    # this replica's share of the global batch
    d_idx = eng.groups.dp_idx
    per = x.shape[0] // dp
    xr, yr = x[d_idx * per:(d_idx + 1) * per], y[d_idx * per:(d_idx + 1) * per]
    for step in range(steps):
        loss = eng.train_step(xr, yr)
        opt.step()
        rl = loss_fn(ref(x), y)
        rl.backward()
        ropt.step()
        ropt.zero_grad()
        if eng.is_last and dp == 1:
            torch.testing.assert_close(loss, rl.detach(), atol=1e-5, rtol=1e-5)
    ref_params = dict(ref.named_parameters(remove_duplicate=False))
    mine = eng.state_dict()
    assert mine, "stage holds no parameters"
    for name, p in mine.items():
        torch.testing.assert_close(p.detach(), ref_params[name].detach(), atol=5e-5, rtol=5e-5, msg=name)


@pytest.mark.parametrize("schedule", ["1f1b", "gpipe"])
def test_pp_gpt_tiny_2stages(schedule):
    run_dist(_w_pp, 2, "gpt", schedule, 1, 4, 2)


def test_pp_gpt_tiny_4stages_1f1b():
    run_dist(_w_pp, 4, "gpt", "1f1b", 1, 4, 2)


def test_dp_pp_2x2_gpt_tiny():
    run_dist(_w_pp, 4, "gpt", "1f1b", 2, 2, 2)


def test_pp_fx_traced_mlp_2stages():
    run_dist(_w_pp, 2, "deep", "1f1b", 1, 2, 2)
