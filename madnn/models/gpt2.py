"""GPT-2 (small .. xl), random init from config — BASELINE config 3:
"GPT-2 medium auto pipeline-parallel, 4 stages over xGMI (P2P microbatching)".

Pre-LN blocks; the second LayerNorm of every block fuses the attention
residual add (one K3 kernel returns both LN(x + a) and x + a).  The LM head is
tied to the token embedding; when the pipeline puts them on different stages
the engine all-reduces the tied gradient between first and last stage
(SURVEY N8).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn

from .. import ops
from ..nn.norm import FusedLayerNorm
from .common import init_module_, SelfAttention, causal_lm_loss, init_normal_, linear, scale_residual_proj_


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    dropout: float = 0.0
    layer_norm_eps: float = 1e-5
    vocab_pad_multiple: int = 64   # embedding/LM-head rows padded (GEMM-friendly, 16-byte rows); loss masks them

    @property
    def padded_vocab(self) -> int:
        m = max(self.vocab_pad_multiple, 1)
        return (self.vocab_size + m - 1) // m * m


_SIZES = {
    "gpt2": dict(n_embd=768, n_layer=12, n_head=12),
    "gpt2-medium": dict(n_embd=1024, n_layer=24, n_head=16),
    "gpt2-large": dict(n_embd=1280, n_layer=36, n_head=20),
    "gpt2-xl": dict(n_embd=1600, n_layer=48, n_head=25),
    "gpt2-tiny": dict(n_embd=64, n_layer=4, n_head=4, vocab_size=512, n_positions=128),
}


def gpt2_config(name: str = "gpt2-medium", **over) -> GPT2Config:
    d = dict(_SIZES[name])
    d.update(over)
    return GPT2Config(**d)


class GPT2Embed(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.wte = nn.Embedding(cfg.padded_vocab, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.n_positions, cfg.n_embd)
        self.drop = nn.Dropout(cfg.dropout)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        if ids.size(1) > self.wpe.num_embeddings:   # host-side: an out-of-range gather faults the GPU
            raise ValueError(f"sequence length {ids.size(1)} exceeds n_positions {self.wpe.num_embeddings}")
        pos = torch.arange(ids.size(1), device=ids.device)
        return self.drop(self.wte(ids) + self.wpe(pos))


class GPT2MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.c_fc = nn.Linear(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = nn.Linear(4 * cfg.n_embd, cfg.n_embd)
        self.drop = nn.Dropout(cfg.dropout)

    def forward(self, x, residual=None):
        """MLP(x) (+ ``residual``, added in c_proj's GEMM epilogue when dropout is off).  Plain
        ``nn.Linear`` layers run as ONE fused autograd node (``ops.gelu_mlp``): the GELU and its
        backward live in the two GEMMs' epilogues."""
        no_drop = self.drop.p == 0.0 or not self.training
        if no_drop and ops.FUSED_LINEAR and type(self.c_fc) is nn.Linear and type(self.c_proj) is nn.Linear:
            return ops.gelu_mlp(x, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias,
                                residual)
        if residual is not None and no_drop:
            return linear(self.c_proj, linear(self.c_fc, x, gelu=True), residual=residual)
        y = self.drop(linear(self.c_proj, linear(self.c_fc, x, gelu=True)))
        return y + residual if residual is not None else y

    def tensor_parallel_pairs(self):
        return [(("c_fc",), "c_proj")]


class GPT2Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln_1 = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.attn = SelfAttention(cfg.n_embd, cfg.n_head, causal=True, dropout=cfg.dropout)
        self.ln_2 = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.mlp = GPT2MLP(cfg)
        self.drop = nn.Dropout(cfg.dropout)

    def forward(self, x):
        y, xr = self.ln_1(x, fork=True)       # xr aliases x: its gradient joins ln_1's backward pass
        a = self.drop(self.attn(y))
        y, h = self.ln_2(a, residual=xr)     # h = x + a, y = LN(h): one kernel
        return self.mlp(y, residual=h)        # h + MLP(y): the add rides in c_proj's GEMM epilogue


class GPT2Head(nn.Module):
    def __init__(self, cfg: GPT2Config, wte: nn.Embedding):
        super().__init__()
        self.ln_f = FusedLayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.lm_head = nn.Linear(cfg.n_embd, cfg.padded_vocab, bias=False)
        self.lm_head.weight = wte.weight      # tied

    def forward(self, x):
        return linear(self.lm_head, self.ln_f(x))


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.config = cfg
        self.embed = GPT2Embed(cfg)
        self.h = nn.ModuleList([GPT2Block(cfg) for _ in range(cfg.n_layer)])
        self.head = GPT2Head(cfg, self.embed.wte)
        init_normal_(self)
        scale_residual_proj_(self.h, ("attn.proj.weight", "mlp.c_proj.weight"), cfg.n_layer)

    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        x = self.embed(ids)
        for blk in self.h:
            x = blk(x)
        return self.head(x)

    @staticmethod
    def init_weights(m: nn.Module):
        init_module_(m)

    def pipeline_layers(self):
        return [self.embed, *self.h, self.head]

    def loss_fn(self, logits, targets, scale: float = 1.0):
        return causal_lm_loss(logits, targets, vocab=self.config.vocab_size, scale=scale)

    def flops_per_token(self) -> float:
        c = self.config
        n = sum(p.numel() for p in self.parameters()) - c.n_positions * c.n_embd
        return 6.0 * n + 12.0 * c.n_layer * c.n_embd * c.n_positions
