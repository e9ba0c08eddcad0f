"""Hugging Face GPT-2 / BERT / Llama through ``madnn.distribute`` on the GPU: the hand-written
kernels are swapped in (K3 LayerNorm/RMSNorm modules, K8 attention via HF's attention
interface) and training tracks an fp32 eager copy of the same model."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _build(kind):
    from madnn.models import hf

    torch.manual_seed(0)
    # head dim 64 / 128 and no dropout: the configurations K8 runs (dropout falls back to SDPA)
    if kind == "gpt2":
        return hf.gpt2_hf("gpt2-tiny", n_embd=256, n_head=4, attn_pdrop=0.0, resid_pdrop=0.0, embd_pdrop=0.0)
    if kind == "bert":
        return hf.bert_hf(hidden_size=256, num_attention_heads=4, intermediate_size=512, hidden_dropout_prob=0.0,
                          attention_probs_dropout_prob=0.0)
    return hf.llama_hf(hidden_size=512, num_attention_heads=4, num_key_value_heads=2, intermediate_size=1024)


@pytest.mark.parametrize("kind", ["gpt2", "bert", "llama"])
def test_hf_model_runs_madnn_kernels(cuda, kind):
    import madnn
    from madnn.nn import FusedLayerNorm, FusedRMSNorm
    from madnn.nn.swap import attention_stats
    from madnn.optim import FusedAdam

    model = _build(kind)
    ref = copy.deepcopy(model).to(cuda).float()
    ropt = torch.optim.AdamW(ref.parameters(), lr=1e-3, weight_decay=0.0)
    opt = FusedAdam(model.parameters(), lr=1e-3, weight_decay=0.0)
    eng, opt = madnn.distribute(model, opt, strategy="dp")
    fused = [m for m in eng.module.modules() if isinstance(m, (FusedLayerNorm, FusedRMSNorm))]
    assert fused, "no K3 norm module was swapped in"
    assert eng.module.config._attn_implementation == "madnn_k8"
    ids = torch.randint(0, 512, (4, 64), generator=torch.Generator().manual_seed(1)).to(cuda)
    loss_fn = madnn.models.hf.hf_loss_fn(eng.module)
    before = attention_stats()["k8"]
    for step in range(3):
        out = eng(ids)
        loss = loss_fn(out.logits, ids)
        loss.backward()
        opt.step()
        rl = loss_fn(ref(ids).logits, ids)
        rl.backward()
        ropt.step()
        ropt.zero_grad()
        assert abs(float(loss.detach()) - float(rl.detach())) < 3e-2 * float(rl.detach()), (kind, step, float(loss.detach()), float(rl.detach()))
    assert attention_stats()["k8"] > before, "attention did not run on K8"
