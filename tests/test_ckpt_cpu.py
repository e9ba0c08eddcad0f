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
