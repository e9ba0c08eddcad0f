"""Spines for Hugging Face ``transformers`` models (module-tree tracer fallback).

HF causal-LM / MLM models are not fx-traceable with torch's plain tracer
(data-dependent control flow, cache objects, mask builders).  The tracer
therefore falls back to the module tree: it finds the repeated block list
(``transformer.h`` for GPT-2, ``model.layers`` for Llama, ``bert.encoder.layer``
for BERT) and wraps embedding -> blocks -> head as single-tensor layers, so
the planner and the pipeline engine treat an HF model like a madnn-zoo one.
Models are built from configs (random init, no download): the GPU box has no
network.  Parity is checked against the HF model's own forward in
tests/test_hf_cpu.py.
"""
from __future__ import annotations

from typing import List, Optional

import torch
from torch import nn

from .common import causal_lm_loss, mlm_loss


def _first(out):
    return out[0] if isinstance(out, (tuple, list)) else out


class _Gpt2Embed(nn.Module):
    def __init__(self, tr):
        super().__init__()
        self.wte, self.wpe, self.drop = tr.wte, tr.wpe, tr.drop

    def forward(self, ids):
        pos = torch.arange(ids.size(1), device=ids.device)[None]
        return self.drop(self.wte(ids) + self.wpe(pos))


class _Gpt2Block(nn.Module):
    def __init__(self, block):
        super().__init__()
        self.block = block

    def forward(self, x):
        return _first(self.block(x))


class _Gpt2Head(nn.Module):
    def __init__(self, model):
        super().__init__()
        self.ln_f, self.lm_head = model.transformer.ln_f, model.lm_head

    def forward(self, x):
        return self.lm_head(self.ln_f(x))


class _LlamaEmbed(nn.Module):
    def __init__(self, m):
        super().__init__()
        self.embed_tokens = m.model.embed_tokens

    def forward(self, ids):
        return self.embed_tokens(ids)


class _LlamaBlock(nn.Module):
    def __init__(self, layer, rotary):
        super().__init__()
        self.layer = layer
        self.rotary = rotary  # one module shared by every block (buffers only)

    def forward(self, x):
        pos = torch.arange(x.size(1), device=x.device)[None]
        pe = self.rotary(x, pos)
        return _first(self.layer(x, attention_mask=None, position_ids=pos, position_embeddings=pe))


class _LlamaHead(nn.Module):
    def __init__(self, m):
        super().__init__()
        self.norm, self.lm_head = m.model.norm, m.lm_head

    def forward(self, x):
        return self.lm_head(self.norm(x))


class _BertEmbed(nn.Module):
    def __init__(self, bert):
        super().__init__()
        self.embeddings = bert.embeddings

    def forward(self, ids):
        return self.embeddings(input_ids=ids)


class _BertLayer(nn.Module):
    def __init__(self, layer):
        super().__init__()
        self.layer = layer

    def forward(self, x):
        return _first(self.layer(x))


class _BertHead(nn.Module):
    def __init__(self, cls):
        super().__init__()
        self.cls = cls

    def forward(self, x):
        out = self.cls(x)
        return out[0] if isinstance(out, tuple) else out


def hf_pipeline_layers(model: nn.Module) -> Optional[List[nn.Module]]:
    """Single-tensor spine for supported HF architectures, else None."""
    name = type(model).__name__
    if name == "GPT2LMHeadModel":
        tr = model.transformer
        return [_Gpt2Embed(tr), *[_Gpt2Block(b) for b in tr.h], _Gpt2Head(model)]
    if name in ("LlamaForCausalLM", "MistralForCausalLM", "Qwen2ForCausalLM"):
        rot = model.model.rotary_emb
        return [_LlamaEmbed(model), *[_LlamaBlock(l, rot) for l in model.model.layers], _LlamaHead(model)]
    if name in ("BertForMaskedLM", "BertForPreTraining"):
        bert = model.bert
        cls = model.cls
        if name == "BertForPreTraining":
            cls = _MLMOnly(model.cls)
        return [_BertEmbed(bert), *[_BertLayer(l) for l in bert.encoder.layer], _BertHead(cls)]
    return None


class _MLMOnly(nn.Module):
    def __init__(self, cls):
        super().__init__()
        self.predictions = cls.predictions

    def forward(self, x):
        return self.predictions(x)


def hf_loss_fn(model: nn.Module):
    name = type(model).__name__
    if name.endswith("ForCausalLM") or name == "GPT2LMHeadModel":
        vocab = model.config.vocab_size
        return lambda logits, targets: causal_lm_loss(logits, targets, vocab=vocab)
    if name.startswith("Bert"):
        vocab = model.config.vocab_size
        return lambda logits, targets: mlm_loss(logits, targets, vocab=vocab)
    return None


def gpt2_hf(size: str = "gpt2-medium", **over):
    from transformers import GPT2Config, GPT2LMHeadModel

    dims = {"gpt2": (768, 12, 12), "gpt2-medium": (1024, 24, 16), "gpt2-large": (1280, 36, 20),
            "gpt2-tiny": (64, 4, 4)}[size]
    kw = dict(n_embd=dims[0], n_layer=dims[1], n_head=dims[2], attn_implementation="sdpa")
    if size == "gpt2-tiny":
        kw.update(vocab_size=512, n_positions=128)
    kw.update(over)
    return GPT2LMHeadModel(GPT2Config(**kw))


def llama_hf(**over):
    from transformers import LlamaConfig, LlamaForCausalLM

    kw = dict(vocab_size=512, hidden_size=64, intermediate_size=160, num_hidden_layers=4, num_attention_heads=4,
              num_key_value_heads=2, max_position_embeddings=256, attn_implementation="sdpa")
    kw.update(over)
    return LlamaForCausalLM(LlamaConfig(**kw))


def bert_hf(**over):
    from transformers import BertConfig, BertForMaskedLM

    kw = dict(vocab_size=512, hidden_size=64, num_hidden_layers=4, num_attention_heads=4, intermediate_size=256,
              max_position_embeddings=128, attn_implementation="sdpa")
    kw.update(over)
    return BertForMaskedLM(BertConfig(**kw))
