"""BERT (base / large) with the masked-LM pretraining head, random init —
BASELINE config 5: "BERT-large auto-partition + activation checkpointing +
fused Adam HIP kernel".

Post-LN encoder: both LayerNorms of every layer are ``LN(x + sublayer(x))``,
i.e. exactly the K3 kernel's fused residual form.  The MLM decoder is tied to
the word embedding.  (The next-sentence head is omitted: synthetic data has
no sentence pairs.)
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import nn

from .. import ops
from ..nn.norm import FusedLayerNorm
from .common import init_module_, SelfAttention, init_normal_, linear, mlm_loss


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 1024
    layers: int = 24
    heads: int = 16
    intermediate: int = 4096
    max_position: int = 512
    type_vocab: int = 2
    dropout: float = 0.0
    layer_norm_eps: float = 1e-12
    vocab_pad_multiple: int = 64

    @property
    def padded_vocab(self) -> int:
        m = max(self.vocab_pad_multiple, 1)
        return (self.vocab_size + m - 1) // m * m


_SIZES = {
    "bert-base": dict(hidden=768, layers=12, heads=12, intermediate=3072),
    "bert-large": dict(hidden=1024, layers=24, heads=16, intermediate=4096),
    "bert-tiny": dict(hidden=64, layers=4, heads=4, intermediate=256, vocab_size=512, max_position=128),
}


def bert_config(name: str = "bert-large", **over) -> BertConfig:
    d = dict(_SIZES[name])
    d.update(over)
    return BertConfig(**d)


class BertEmbed(nn.Module):
    def __init__(self, cfg: BertConfig):
        super().__init__()
        self.word = nn.Embedding(cfg.padded_vocab, cfg.hidden)
        self.position = nn.Embedding(cfg.max_position, cfg.hidden)
        self.token_type = nn.Embedding(cfg.type_vocab, cfg.hidden)
        self.norm = FusedLayerNorm(cfg.hidden, eps=cfg.layer_norm_eps)
        self.drop = nn.Dropout(cfg.dropout)

    def forward(self, ids):
        if ids.size(1) > self.position.num_embeddings:   # host-side: an out-of-range gather faults the GPU
            raise ValueError(f"sequence length {ids.size(1)} exceeds max_position {self.position.num_embeddings}")
        pos = torch.arange(ids.size(1), device=ids.device)
        # single-segment synthetic input: token type 0 for every position
        x = self.word(ids) + (self.position(pos) + self.token_type.weight[0])
        return self.drop(self.norm(x))


class BertLayer(nn.Module):
    def __init__(self, cfg: BertConfig):
        super().__init__()
        self.attn = SelfAttention(cfg.hidden, cfg.heads, causal=False, dropout=cfg.dropout)
        self.attn_norm = FusedLayerNorm(cfg.hidden, eps=cfg.layer_norm_eps)
        self.fc1 = nn.Linear(cfg.hidden, cfg.intermediate)
        self.fc2 = nn.Linear(cfg.intermediate, cfg.hidden)
        self.ffn_norm = FusedLayerNorm(cfg.hidden, eps=cfg.layer_norm_eps)
        self.drop = nn.Dropout(cfg.dropout)

    def tensor_parallel_pairs(self):
        return [(("fc1",), "fc2")]

    def forward(self, x):
        fused = (self.drop.p == 0.0 or not self.training) and ops.FUSED_LINEAR
        if fused and type(self.attn) is SelfAttention:
            # LN(x + attn(x)): x's residual gradient is summed inside the QKV projection's data-gradient
            # GEMM (ops.linear_tee), not by a separate pass over x's two gradients
            a, xr = self.attn.forward_tee(x)
            y, _ = self.attn_norm(a, residual=xr)
        else:
            y, _ = self.attn_norm(self.drop(self.attn(x)), residual=x)
        if fused and type(self.fc1) is nn.Linear and type(self.fc2) is nn.Linear:
            # one fused autograd node: the exact GELU and its backward in the two GEMMs' epilogues, the
            # residual y added in fc2's epilogue and its gradient inside y's data-gradient GEMM
            h = ops.gelu_mlp(y, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, residual=y,
                             approximate="none")
            return self.ffn_norm(h)
        h = self.drop(linear(self.fc2, F.gelu(linear(self.fc1, y))))
        z, _ = self.ffn_norm(h, residual=y)
        return z


class BertMLMHead(nn.Module):
    def __init__(self, cfg: BertConfig, word: nn.Embedding):
        super().__init__()
        self.dense = nn.Linear(cfg.hidden, cfg.hidden)
        self.norm = FusedLayerNorm(cfg.hidden, eps=cfg.layer_norm_eps)
        self.decoder = nn.Linear(cfg.hidden, cfg.padded_vocab, bias=True)
        self.decoder.weight = word.weight  # tied

    def forward(self, x):
        return linear(self.decoder, self.norm(F.gelu(linear(self.dense, x))))


class BertForPreTraining(nn.Module):
    def __init__(self, cfg: BertConfig):
        super().__init__()
        self.config = cfg
        self.embed = BertEmbed(cfg)
        self.layers = nn.ModuleList([BertLayer(cfg) for _ in range(cfg.layers)])
        self.head = BertMLMHead(cfg, self.embed.word)
        init_normal_(self)

    def forward(self, ids):
        x = self.embed(ids)
        for layer in self.layers:
            x = layer(x)
        return self.head(x)

    @staticmethod
    def init_weights(m: nn.Module):
        init_module_(m)

    def pipeline_layers(self):
        return [self.embed, *self.layers, self.head]

    def loss_fn(self, logits, targets, scale: float = 1.0):
        return mlm_loss(logits, targets, vocab=self.config.vocab_size, scale=scale)
