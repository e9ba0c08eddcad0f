"""Llama-3 (8B and scaled-down variants), random init — BASELINE config 4:
"Llama-3 8B auto hybrid DPxPP on 8xMI355X (288 GB HBM per-GPU sizing)".

Pre-RMSNorm blocks, grouped-query attention (32 query / 8 KV heads at 8B),
RoPE (theta 500k, host-precomputed tables), SwiGLU MLP with the gate and up
projections fused into one GEMM.  The post-attention RMSNorm fuses the
residual add (K3 kernel).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

from .. import ops
from ..nn.norm import FusedRMSNorm
from .common import init_module_, RotaryEmbedding, SelfAttention, causal_lm_loss, init_normal_, linear


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden: int = 4096
    intermediate: int = 14336
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    rope_theta: float = 500000.0
    max_position: int = 8192
    rms_eps: float = 1e-5


_SIZES = {
    "llama3-8b": dict(),
    "llama3-70b": dict(hidden=8192, intermediate=28672, layers=80, heads=64, kv_heads=8),
    "llama3-1b": dict(hidden=2048, intermediate=8192, layers=16, heads=32, kv_heads=8),
    "llama3-tiny": dict(vocab_size=512, hidden=64, intermediate=160, layers=4, heads=4, kv_heads=2,
                        max_position=256),
}


def llama_config(name: str = "llama3-8b", **over) -> LlamaConfig:
    d = dict(_SIZES[name])
    d.update(over)
    return LlamaConfig(**d)


class LlamaEmbed(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden)

    def forward(self, ids):
        return self.embed_tokens(ids)


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.inter = cfg.intermediate
        self.gate_up = nn.Linear(cfg.hidden, 2 * cfg.intermediate, bias=False)
        self.down = nn.Linear(cfg.intermediate, cfg.hidden, bias=False)

    def forward(self, x, residual=None):
        """down(silu(g) * u) (+ ``residual``, added in the down projection's GEMM epilogue); the
        SwiGLU is one K15 pass each way on the GPU."""
        return linear(self.down, ops.swiglu(linear(self.gate_up, x)), residual=residual)


class LlamaBlock(nn.Module):
    def __init__(self, cfg: LlamaConfig, rope: RotaryEmbedding):
        super().__init__()
        self.input_norm = FusedRMSNorm(cfg.hidden, eps=cfg.rms_eps)
        self.attn = SelfAttention(cfg.hidden, cfg.heads, cfg.kv_heads, bias=False, causal=True, rope=rope)
        self.post_attn_norm = FusedRMSNorm(cfg.hidden, eps=cfg.rms_eps)
        self.mlp = LlamaMLP(cfg)

    def forward(self, x):
        y, xr = self.input_norm(x, fork=True)  # residual path's gradient joins the norm's backward
        a = self.attn(y)
        y, h = self.post_attn_norm(a, residual=xr)
        return self.mlp(y, residual=h)


class LlamaHead(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.norm = FusedRMSNorm(cfg.hidden, eps=cfg.rms_eps)
        self.lm_head = nn.Linear(cfg.hidden, cfg.vocab_size, bias=False)

    def forward(self, x):
        return linear(self.lm_head, self.norm(x))


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.config = cfg
        rope = RotaryEmbedding(cfg.hidden // cfg.heads, cfg.rope_theta, cfg.max_position)
        self.embed = LlamaEmbed(cfg)
        self.layers = nn.ModuleList([LlamaBlock(cfg, rope) for _ in range(cfg.layers)])
        self.head = LlamaHead(cfg)
        init_normal_(self)

    def forward(self, ids):
        x = self.embed(ids)
        for blk in self.layers:
            x = blk(x)
        return self.head(x)

    @staticmethod
    def init_weights(m: nn.Module):
        init_module_(m)

    def pipeline_layers(self):
        return [self.embed, *self.layers, self.head]

    def loss_fn(self, logits, targets, scale: float = 1.0):
        return causal_lm_loss(logits, targets, vocab=self.config.vocab_size, scale=scale)
