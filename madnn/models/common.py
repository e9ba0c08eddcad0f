"""Shared transformer pieces.

Attention on the GPU is madnn's K8 MFMA flash-attention kernel, reading the packed
QKV projection in place ([B, S, heads, D], no transposes); elsewhere (CPU, dropout,
other head dims) ``F.scaled_dot_product_attention``.  QKV is one fused projection
GEMM (hipBLASLt); norms are the madnn K3 kernel with the residual add fused in.

Every transformer in the zoo exposes ``pipeline_layers()``: a list of modules
whose sequential composition equals ``forward`` (embedding -> blocks -> head),
each taking and returning ONE tensor.  That is the spine the planner
partitions into pipeline stages.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import nn

from .. import ops


def causal_lm_loss(logits: torch.Tensor, targets: torch.Tensor, vocab: int = None, scale: float = 1.0) -> torch.Tensor:
    """Next-token cross entropy (shifted), fp32 math; on the GPU one fused K6 kernel
    each way over the bf16 logits (no fp32 copy, no slicing copies).  ``scale``: a microbatched
    step's 1 / M (``ops.scaled_loss``)."""
    from .. import ops

    return ops.cross_entropy(logits, targets, shift=True, vocab=vocab, scale=scale)


def mlm_loss(logits: torch.Tensor, targets: torch.Tensor, vocab: int = None, scale: float = 1.0) -> torch.Tensor:
    from .. import ops

    return ops.cross_entropy(logits, targets, shift=False, vocab=vocab, ignore_index=-100, scale=scale)


def linear(mod: nn.Module, x: torch.Tensor, gelu: bool = False, residual: torch.Tensor = None) -> torch.Tensor:
    """``mod(x)`` (then tanh-GELU if asked).  A plain ``nn.Linear`` runs through ``ops.linear``,
    whose backward produces the bias gradient (and the GELU backward) in one K11 pass and writes
    the weight gradient straight into the data-parallel bucket; any other module (e.g. a
    tensor-parallel replacement) is called as is."""
    if ops.FUSED_LINEAR and type(mod) is nn.Linear:
        return ops.linear(x, mod.weight, mod.bias, gelu=gelu, residual=residual)
    y = mod(x)
    y = F.gelu(y, approximate="tanh") if gelu else y
    return y + residual if residual is not None else y


class SelfAttention(nn.Module):
    """Multi-head (optionally grouped-query) self-attention with one QKV GEMM."""

    def __init__(self, hidden: int, heads: int, kv_heads: int = None, bias: bool = True, causal: bool = True,
                 dropout: float = 0.0, rope=None):
        super().__init__()
        self.hidden, self.heads = hidden, heads
        self.kv_heads = kv_heads or heads
        self.head_dim = hidden // heads
        self.causal, self.dropout, self.rope = causal, dropout, rope
        self.qkv = nn.Linear(hidden, (heads + 2 * self.kv_heads) * self.head_dim, bias=bias)
        self.proj = nn.Linear(heads * self.head_dim, hidden, bias=bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b, s, _ = x.shape
        return self.attend(linear(self.qkv, x), b, s)

    def forward_tee(self, x: torch.Tensor):
        """``(attn(x), x')``: the QKV projection through :func:`ops.linear_tee`, so a residual path
        that uses ``x'`` has its gradient summed inside the projection's data-gradient GEMM."""
        b, s, _ = x.shape
        if ops.FUSED_LINEAR and type(self.qkv) is nn.Linear:
            qkv, xr = ops.linear_tee(x, self.qkv.weight, self.qkv.bias)
            return self.attend(qkv, b, s), xr
        return self.forward(x), x

    def attend(self, qkv: torch.Tensor, b: int, s: int) -> torch.Tensor:
        """Attention and the output projection on the QKV projection's output ``[b, s, (H + 2 Hkv) D]``."""
        qkv = qkv.view(b, s, self.heads + 2 * self.kv_heads, self.head_dim)
        drop = self.dropout if self.training else 0.0
        if ops.attention_supported(qkv, self.head_dim, drop):
            # K8 HIP attention on the [B, S, heads, D] layout the projection produced: no
            # transposes; it reads q/k/v and writes dQKV in place
            if self.rope is not None:
                # K14: q and k rotated in one pass into a packed buffer (backward: in place on dQKV)
                qkv = ops.rope_qkv(qkv.contiguous(), self.rope.cos, self.rope.sin, self.heads + self.kv_heads)
            o = ops.attention_qkvpacked(qkv, self.heads, self.kv_heads, causal=self.causal)
            return linear(self.proj, o.view(b, s, self.heads * self.head_dim))
        q, k, v = qkv.split([self.heads, self.kv_heads, self.kv_heads], dim=2)
        q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        if self.rope is not None:
            q, k = self.rope(q, k)
        gqa = self.kv_heads != self.heads
        o = F.scaled_dot_product_attention(q, k, v, is_causal=self.causal,
                                           dropout_p=self.dropout if self.training else 0.0, enable_gqa=gqa)
        return linear(self.proj, o.transpose(1, 2).reshape(b, s, self.heads * self.head_dim))


class RotaryEmbedding(nn.Module):
    """RoPE with a host-precomputed cos/sin table (no on-device trig per element:
    cdna_hip_programming.md Appendix B, "Element-wise")."""

    def __init__(self, head_dim: int, theta: float = 10000.0, max_pos: int = 8192):
        super().__init__()
        self.head_dim, self.theta, self.max_pos = head_dim, theta, max_pos
        cos, sin = self._tables(torch.device("cpu") if torch.empty(0).device.type == "meta" else None)
        self.register_buffer("cos", cos, persistent=False)
        self.register_buffer("sin", sin, persistent=False)

    def _tables(self, device=None):
        inv = 1.0 / (self.theta ** (torch.arange(0, self.head_dim, 2, dtype=torch.float64, device=device)
                                    / self.head_dim))
        t = torch.arange(self.max_pos, dtype=torch.float64, device=device)
        f = torch.outer(t, inv)
        return torch.cat([f.cos(), f.cos()], -1).float(), torch.cat([f.sin(), f.sin()], -1).float()

    def reset_parameters(self):
        """Recompute the tables (after ``to_empty`` materialisation from the meta device)."""
        cos, sin = self._tables(self.cos.device)
        self.cos.copy_(cos)
        self.sin.copy_(sin)

    def _apply(self, fn, *args, **kwargs):
        # a module-wide dtype cast (model.bfloat16()) must not round the tables: K14 reads them in
        # fp32 (recomputed exactly on the tables' device, never converted back from bf16)
        super()._apply(fn, *args, **kwargs)
        if self.cos.dtype != torch.float32 and self.cos.device.type != "meta":
            self.cos, self.sin = self._tables(self.cos.device)
        return self

    @staticmethod
    def _rot(x):
        x1, x2 = x.chunk(2, dim=-1)
        return torch.cat([-x2, x1], dim=-1)

    def forward(self, q, k, seq_dim: int = -2):
        """q/k as [B, heads, S, D] (``seq_dim=-2``) or [B, S, heads, D] (``seq_dim=1``)."""
        s = q.size(seq_dim)
        cos = self.cos[:s].to(q.dtype)
        sin = self.sin[:s].to(q.dtype)
        if seq_dim == 1:
            cos, sin = cos[:, None, :], sin[:, None, :]
        return q * cos + self._rot(q) * sin, k * cos + self._rot(k) * sin


def init_module_(m: nn.Module, std: float = 0.02):
    """Initialise ONE module's own tensors (used when materialising from the meta device)."""
    with torch.no_grad():
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, std)
        elif hasattr(m, "reset_parameters") and not isinstance(m, (nn.Linear, nn.Embedding)):
            if not any(True for _ in m.children()):
                m.reset_parameters()


def init_normal_(module: nn.Module, std: float = 0.02):
    for m in module.modules():
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, std)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, std)


def scale_residual_proj_(blocks, names, n_layer: int, std: float = 0.02):
    """GPT-2 style 1/sqrt(2L) init of residual output projections."""
    for blk in blocks:
        for n, p in blk.named_parameters():
            if any(n.endswith(x) for x in names):
                nn.init.normal_(p, 0.0, std / math.sqrt(2 * n_layer))
