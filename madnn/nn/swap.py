"""Put madnn's hand-written gfx950 kernels under an ARBITRARY model.

``distribute()`` calls :func:`use_madnn_kernels` on the model before tracing it,
so a Hugging Face GPT-2 / BERT / Llama (or any torch model) trains on the same
kernels as madnn's zoo, not only on the fused optimizer and bucket kernels:

* ``nn.LayerNorm``          -> :class:`FusedLayerNorm` (K3, fp32 statistics);
* ``*RMSNorm`` (HF Llama)   -> :class:`FusedRMSNorm` (K3 RMS variant);
* ``nn.BatchNorm2d``        -> :class:`FusedBatchNorm2d` (K5 NHWC kernels on
  channels_last activations, eager elsewhere);
* Hugging Face attention    -> the K8 MFMA flash-attention kernel, registered as
  the ``"madnn_k8"`` attention implementation (HF's ``AttentionInterface``):
  unmasked (or causal-only) bf16 attention with head dim 64/128 runs K8 straight
  from HF's [B, H, S, D] views; padding masks, dropout, position biases and
  decoding fall back to HF's SDPA path.

Every swap keeps parameter and buffer names (state dicts interchange with the
original model).  The reference had no kernels of its own at all.
"""
from __future__ import annotations

from typing import Dict

import torch
from torch import nn

from .. import ops
from .norm import FusedBatchNorm2d, FusedLayerNorm, FusedRMSNorm

ATTN_IMPL = "madnn_k8"
_registered = {"done": False}


def _is_rmsnorm(m: nn.Module) -> bool:
    if isinstance(m, FusedRMSNorm) or not type(m).__name__.endswith("RMSNorm"):
        return False
    w = getattr(m, "weight", None)
    eps = getattr(m, "variance_epsilon", getattr(m, "eps", None))
    return isinstance(w, nn.Parameter) and w.dim() == 1 and eps is not None and not list(m.children())


def _swap(model: nn.Module, counts: Dict[str, int]) -> None:
    for name, child in list(model.named_children()):
        new = None
        if type(child) is nn.LayerNorm and len(child.normalized_shape) == 1 and child.elementwise_affine \
                and ops.hidden_supported(child.normalized_shape[0]):
            new = FusedLayerNorm(child.normalized_shape, child.eps, bias=child.bias is not None,
                                 device=child.weight.device, dtype=child.weight.dtype)
            key = "layernorm"
        elif _is_rmsnorm(child) and ops.hidden_supported(child.weight.numel()):
            eps = getattr(child, "variance_epsilon", getattr(child, "eps", 1e-6))
            new = FusedRMSNorm(child.weight.numel(), eps=float(eps), device=child.weight.device,
                               dtype=child.weight.dtype)
            key = "rmsnorm"
        elif type(child) is nn.BatchNorm2d:
            dev = child.running_mean.device if child.track_running_stats else None
            new = FusedBatchNorm2d(child.num_features, child.eps, child.momentum, child.affine,
                                   child.track_running_stats, device=dev)
            key = "batchnorm"
        if new is None:
            _swap(child, counts)
            continue
        # adopt the original tensors themselves (no copy; works on the meta device too)
        new.load_state_dict(child.state_dict(), strict=True, assign=True)
        new.train(child.training)
        setattr(model, name, new)
        counts[key] = counts.get(key, 0) + 1


def madnn_attention_forward(module, query, key, value, attention_mask, dropout: float = 0.0, scaling=None,
                            is_causal=None, position_bias=None, **kwargs):
    """HF attention-interface entry: K8 for what it supports, HF SDPA for the rest."""
    is_causal = is_causal if is_causal is not None else getattr(module, "is_causal", True)
    q_len, kv_len = query.shape[2], key.shape[2]
    if (attention_mask is None and position_bias is None and dropout == 0.0 and q_len == kv_len
            and not kwargs.get("output_attentions", False)
            and ops.attention_supported(query, query.shape[-1]) and key.dtype == query.dtype):
        o = ops.attention(query.transpose(1, 2), key.transpose(1, 2), value.transpose(1, 2),
                          causal=bool(is_causal and q_len > 1), scale=scaling)
        _stats["k8"] += 1
        return o, None
    from transformers.integrations.sdpa_attention import sdpa_attention_forward

    _stats["sdpa"] += 1
    return sdpa_attention_forward(module, query, key, value, attention_mask, dropout=dropout, scaling=scaling,
                                  is_causal=is_causal, position_bias=position_bias, **kwargs)


_stats = {"k8": 0, "sdpa": 0}


def attention_stats() -> Dict[str, int]:
    """How many HF attention calls ran K8 vs fell back to SDPA (diagnostics / tests)."""
    return dict(_stats)


def register_hf_attention() -> bool:
    if _registered["done"]:
        return True
    try:
        from transformers import AttentionInterface
        from transformers.masking_utils import AttentionMaskInterface, sdpa_mask
    except Exception:  # noqa: BLE001 - transformers absent or too old: nothing to route
        return False
    AttentionInterface.register(ATTN_IMPL, madnn_attention_forward)
    AttentionMaskInterface.register(ATTN_IMPL, sdpa_mask)
    _registered["done"] = True
    return True


def _route_hf_attention(model: nn.Module) -> int:
    cfg = getattr(model, "config", None)
    if cfg is None or not hasattr(cfg, "_attn_implementation") or not register_hf_attention():
        return 0
    n = 0
    for m in model.modules():
        c = getattr(m, "config", None)
        if c is not None and hasattr(c, "_attn_implementation"):
            try:
                c._attn_implementation = ATTN_IMPL
            except Exception:  # noqa: BLE001
                c._attn_implementation_internal = ATTN_IMPL
            n += 1
    return n


def use_madnn_kernels(model: nn.Module) -> Dict[str, int]:
    """Swap in madnn's kernels (see module doc) in place; returns what was swapped."""
    counts: Dict[str, int] = {}
    _swap(model, counts)
    if _route_hf_attention(model):
        counts["hf_attention"] = 1
    return counts
