"""Model-level GPU checks for the transformer zoo on the HIP kernels (K3 norms, K6 cross-entropy,
K8 attention): causal models must not see the future, and the fused shifted LM loss must equal
the plain shifted cross-entropy of the same logits."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _models():
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.models.llama import Llama, llama_config

    return {
        # head dim 64 so K8 attention runs (RoPE + grouped-query heads for Llama)
        "gpt2": lambda: GPT2(gpt2_config("gpt2-tiny", n_embd=256, n_head=4, n_layer=2, dropout=0.0,
                                          n_positions=256)),
        "llama": lambda: Llama(llama_config("llama3-tiny", hidden=256, heads=4, kv_heads=2, intermediate=512,
                                            layers=2)),
        # head dim 128, one KV head (the 8B model's head size)
        "llama_d128": lambda: Llama(llama_config("llama3-tiny", hidden=512, heads=4, kv_heads=1, intermediate=512,
                                                 layers=2)),
    }


@pytest.mark.parametrize("seq", [96, 192])   # ragged key tiles / whole 64-key tiles (DMA-ring forward)
@pytest.mark.parametrize("name", ["gpt2", "llama", "llama_d128"])
def test_causal_lm_does_not_see_the_future(cuda, name, seq):
    torch.manual_seed(0)
    model = _models()[name]().to(cuda).bfloat16().eval()
    vocab = model.config.vocab_size
    ids = torch.randint(0, vocab, (2, seq), device=cuda)
    t = seq * 3 // 4 - 2
    ids2 = ids.clone()
    ids2[:, t:] = (ids2[:, t:] + 1 + torch.randint(0, vocab - 1, ids2[:, t:].shape, device=cuda)) % vocab
    with torch.no_grad():
        a, b = model(ids).float(), model(ids2).float()
    torch.testing.assert_close(a[:, :t], b[:, :t], atol=1e-3, rtol=0)
    assert (a[:, t:] - b[:, t:]).abs().max().item() > 1e-2


def test_causal_lm_training_mode_no_leak_d128(cuda):
    """Training mode, gradients on, the Llama-3 8B head size (D = 128, GQA) at S = 1024: with the
    tokens from t on replaced, the logits before t, the prefix loss and its gradient with respect
    to the embeddings before t are unchanged, and that gradient is exactly zero at positions >= t
    (no key or value of the future receives gradient from the past's loss)."""
    from madnn.models.llama import Llama, llama_config

    torch.manual_seed(7)
    model = Llama(llama_config("llama3-tiny", hidden=1024, heads=8, kv_heads=2, intermediate=1024, layers=2,
                               max_position=2048)).to(cuda).bfloat16().train()
    vocab = model.config.vocab_size
    S, t = 1024, 700
    ids = torch.randint(0, vocab, (2, S), device=cuda)
    ids2 = ids.clone()
    ids2[:, t:] = (ids2[:, t:] + 1 + torch.randint(0, vocab - 1, ids2[:, t:].shape, device=cuda)) % vocab
    outs = []
    for x in (ids, ids2):
        cap = {}

        def keep(_m, _i, o):   # returns None: the output itself is not replaced
            o.retain_grad()
            cap["e"] = o

        h = model.embed.register_forward_hook(keep)
        try:
            logits = model(x)
        finally:
            h.remove()
        loss = F.cross_entropy(logits[:, : t - 1].float().reshape(-1, vocab), x[:, 1:t].reshape(-1))
        loss.backward()
        outs.append((logits.detach().float(), loss.detach(), cap["e"].grad.detach().float()))
        model.zero_grad(set_to_none=True)
    (la, lossa, ga), (lb, lossb, gb) = outs
    torch.testing.assert_close(la[:, :t], lb[:, :t], atol=1e-3, rtol=0)
    torch.testing.assert_close(lossa, lossb, atol=1e-5, rtol=0)
    assert ga[:, :t].abs().max() > 0
    torch.testing.assert_close(ga[:, :t], gb[:, :t], atol=1e-4, rtol=0)
    assert ga[:, t:].abs().max().item() == 0.0 and gb[:, t:].abs().max().item() == 0.0
    assert (la[:, t:] - lb[:, t:]).abs().max().item() > 1e-2


@pytest.mark.parametrize("name", ["gpt2", "llama", "llama_d128"])
def test_fused_lm_loss_is_shifted_cross_entropy(cuda, name):
    torch.manual_seed(1)
    model = _models()[name]().to(cuda).bfloat16()
    vocab = model.config.vocab_size
    ids = torch.randint(0, vocab, (2, 64), device=cuda)
    logits = model(ids)
    loss = model.loss_fn(logits, ids)
    ref = F.cross_entropy(logits[:, :-1, :vocab].float().reshape(-1, vocab), ids[:, 1:].reshape(-1))
    torch.testing.assert_close(loss.detach().float(), ref.detach(), atol=2e-3, rtol=2e-3)
