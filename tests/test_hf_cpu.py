"""Hugging Face models through madnn: spine parity with the HF forward, and a
2-stage pipeline run on CPU/gloo (models from configs, random init, no download)."""
import copy

import pytest
import torch

from dist_utils import run_dist

transformers = pytest.importorskip("transformers")


@pytest.mark.parametrize("kind", ["gpt2", "llama", "bert"])
def test_hf_spine_matches_model(kind):
    from madnn.models import hf
    from madnn.planner.trace import run_spine, trace

    torch.manual_seed(0)
    m = {"gpt2": lambda: hf.gpt2_hf("gpt2-tiny"), "llama": hf.llama_hf, "bert": hf.bert_hf}[kind]().eval()
    sp = trace(m)
    assert sp.source == "hf" and len(sp) == 6
    ids = torch.randint(0, 512, (2, 16))
    with torch.no_grad():
        ref = m(input_ids=ids).logits
        out = run_spine(sp, ids)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)


def _w_hf_pp(rank, world):
    import madnn
    from madnn.models import hf
    from madnn.optim import FusedAdam

    torch.manual_seed(0)
    m = hf.llama_hf()
    ref = copy.deepcopy(m)
    opt = FusedAdam(m.parameters(), lr=1e-3)
    ids = torch.randint(0, 512, (4, 16), generator=torch.Generator().manual_seed(1))
    eng, opt = madnn.distribute(m, opt, strategy="pp", pp_stages=2, microbatches=2, example_input=ids[:1],
                                checkpointing="none")
    loss = eng.train_step(ids, ids)
    opt.step()
    if eng.is_last:
        rl = hf.hf_loss_fn(ref)(ref(input_ids=ids).logits, ids)
        torch.testing.assert_close(loss, rl.detach(), atol=1e-5, rtol=1e-5)
    names = set(eng.state_dict())
    assert names and names <= set(dict(ref.named_parameters()).keys())


@pytest.mark.slow
def test_hf_llama_pipeline_2_stages():
    run_dist(_w_hf_pp, 2)
