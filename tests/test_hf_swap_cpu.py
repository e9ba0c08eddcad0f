"""use_madnn_kernels on Hugging Face models (CPU tier: module swaps and numerics of the
eager fallbacks; the GPU tier runs the same models on the HIP kernels)."""
import copy

import pytest
import torch

from madnn.models import hf
from madnn.nn import FusedBatchNorm2d, FusedLayerNorm, FusedRMSNorm, use_madnn_kernels


@pytest.mark.parametrize("build,kinds", [(hf.gpt2_hf, {"layernorm"}), (hf.bert_hf, {"layernorm"}),
                                          (hf.llama_hf, {"rmsnorm"})])
def test_swap_keeps_outputs_and_state_dict(build, kinds):
    torch.manual_seed(0)
    m = build(**({"size": "gpt2-tiny"} if build is hf.gpt2_hf else {})) if build is not hf.gpt2_hf else build("gpt2-tiny")
    m.eval()
    ref = copy.deepcopy(m)
    sd_keys = set(ref.state_dict())
    counts = use_madnn_kernels(m)
    assert kinds <= set(counts) and counts.get("hf_attention") == 1
    assert set(m.state_dict()) == sd_keys
    assert any(isinstance(x, (FusedLayerNorm, FusedRMSNorm)) for x in m.modules())
    assert m.config._attn_implementation == "madnn_k8"
    ids = torch.randint(0, 512, (2, 16))
    with torch.no_grad():
        a = m(ids).logits
        b = ref(ids).logits
    torch.testing.assert_close(a, b, atol=2e-5, rtol=2e-5)


def test_swap_batchnorm_and_meta():
    from torch import nn

    m = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.ReLU())
    m[1].running_mean.fill_(0.5)
    use_madnn_kernels(m)
    assert isinstance(m[1], FusedBatchNorm2d) and float(m[1].running_mean[0]) == 0.5
    with torch.device("meta"):
        mm = nn.Sequential(nn.Linear(64, 64), nn.LayerNorm(64))
    use_madnn_kernels(mm)
    assert isinstance(mm[1], FusedLayerNorm) and mm[1].weight.is_meta
