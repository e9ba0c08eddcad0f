"""Flat parameter space: a model's parameters re-homed into a few flat buckets.

This is the memory layout every engine and the fused optimizers share
(MI355X-first replacement for Torch7 ``getParameters()`` flattening,
cifar_example/sgd-torchad_nn-cifar.lua:109, and the per-tensor loops of
datamodule.lua:211-224):

* parameters are VIEWS into one ``model`` buffer per bucket, in the compute
  dtype (bf16 by default; norm layers may stay fp32 in their own buckets);
* each bucket owns an fp32 ``master`` copy (aliased to ``model`` when the
  compute dtype is already fp32) that the fused optimizer updates and then
  writes back to ``model`` in the same kernel — no separate cast pass;
* each bucket owns a ``grad`` buffer (reduce dtype) that the K4 pack kernel
  fills from ``p.grad`` with the 1/W average fused in, and that RCCL reduces
  in place;
* conv weights can be laid out channels_last inside the flat buffer, so a
  channels_last network never re-layouts its weights per forward;
* every tensor starts on a 16-element boundary so the K4/K1/K2 kernels use
  16-byte vector accesses throughout.

Sized for 288 GB HBM3E per GPU: buckets are large (64 MB by default) so the
all-reduce runs as few, large RCCL calls spread over the 7 xGMI links.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence

import torch
from torch import nn

from .. import ops
from ..ops import native_runtime
from ..ops.reference import is_dense

ALIGN = 16


def _phys_view(flat_slice: torch.Tensor, shape, channels_last: bool) -> torch.Tensor:
    """A tensor of logical ``shape`` backed by ``flat_slice`` in physical order."""
    if channels_last and len(shape) == 4:
        n, c, h, w = shape
        return flat_slice.view(n, h, w, c).permute(0, 3, 1, 2)
    return flat_slice.view(shape)


class FlatBucket:
    def __init__(self, index: int, dtype: torch.dtype, group_id: int):
        self.index = index
        self.dtype = dtype
        self.group_id = group_id
        self.params: List[nn.Parameter] = []
        self.offsets: List[int] = []
        self.numel = 0
        self.model: Optional[torch.Tensor] = None
        self.master: Optional[torch.Tensor] = None
        self.grad: Optional[torch.Tensor] = None
        # reducer bookkeeping
        self.pending = 0
        self.launched = False
        self.work = None
        self.event = None

    @property
    def has_master_copy(self) -> bool:
        return self.master is not None and self.master.data_ptr() != self.model.data_ptr()

    def __repr__(self):
        return f"FlatBucket(#{self.index}, {self.dtype}, {len(self.params)} params, {self.numel} elems)"


class FlatParamSpace:
    """Owns every trainable parameter of a module as views into flat buckets."""

    def __init__(self, param_groups: Sequence[Sequence[nn.Parameter]], *,
                 dtype_of: Callable[[nn.Parameter], torch.dtype],
                 bucket_cap_mb: float = 64.0,
                 reduce_dtype: torch.dtype = torch.float32,
                 channels_last_of: Optional[Callable[[nn.Parameter], bool]] = None,
                 device: Optional[torch.device] = None):
        self.reduce_dtype = reduce_dtype
        self.buckets: List[FlatBucket] = []
        self.param_info: Dict[int, tuple] = {}  # id(p) -> (bucket, offset, channels_last)
        self.group_of_param: Dict[int, int] = {}
        cap_elems = int(bucket_cap_mb * 1024 * 1024 / torch.tensor([], dtype=reduce_dtype).element_size())
        cl_of = channels_last_of or (lambda p: False)
        for gi, group in enumerate(param_groups):
            plist = [p for p in group if p.requires_grad]
            # backward readiness is roughly reverse registration order
            plist = list(reversed(plist))
            by_dtype: Dict[torch.dtype, List[nn.Parameter]] = {}
            for p in plist:
                by_dtype.setdefault(dtype_of(p), []).append(p)
            for dt, ps in by_dtype.items():
                bucket_of, offset_of, sizes = native_runtime.plan_buckets([p.numel() for p in ps], cap_elems, ALIGN)
                base = len(self.buckets)
                for k in range(len(sizes)):
                    self.buckets.append(FlatBucket(base + k, dt, gi))
                for p, b, off in zip(ps, bucket_of, offset_of):
                    bk = self.buckets[base + b]
                    bk.params.append(p)
                    bk.offsets.append(off)
                    self.group_of_param[id(p)] = gi
                for k, sz in enumerate(sizes):
                    self.buckets[base + k].numel = int(sz)
        for bk in self.buckets:
            self._materialize(bk, device, cl_of)

    def _materialize(self, bk: FlatBucket, device, cl_of):
        dev = device or bk.params[0].device
        master = torch.zeros(bk.numel, dtype=torch.float32, device=dev)
        for p, off in zip(bk.params, bk.offsets):
            cl = bool(cl_of(p)) and p.dim() == 4
            _phys_view(master[off:off + p.numel()], p.shape, cl).copy_(p.detach())
            self.param_info[id(p)] = (bk, off, cl)
        if bk.dtype == torch.float32:
            model = master
        else:
            model = master.to(bk.dtype)
        for p, off in zip(bk.params, bk.offsets):
            cl = self.param_info[id(p)][2]
            p.data = _phys_view(model[off:off + p.numel()], p.shape, cl)
            # an existing p.grad stays valid: pack_grads re-layouts it if its strides differ
        bk.model = model
        bk.master = master

    # ------------------------------------------------------------------ grads
    def grad_buffer(self, bk: FlatBucket) -> torch.Tensor:
        if bk.grad is None:
            bk.grad = torch.zeros(bk.numel, dtype=self.reduce_dtype, device=bk.model.device)
        return bk.grad

    def bucket_grads(self, bk: FlatBucket):
        """(tensors, offsets) of the params of ``bk`` that currently hold a grad."""
        ts, offs = [], []
        for p, off in zip(bk.params, bk.offsets):
            g = p.grad
            if g is None:
                continue
            if g.stride() != p.stride() or not is_dense(g):
                g = torch.empty_like(p).copy_(g)  # match the bucket's physical layout
            ts.append(g)
            offs.append(off)
        return ts, offs

    def pack_grads(self, bk: FlatBucket, scale: float = 1.0) -> torch.Tensor:
        buf = self.grad_buffer(bk)
        ts, offs = self.bucket_grads(bk)
        if len(ts) < len(bk.params):
            buf.zero_()  # params without grad contribute zeros (unused in this step)
        ops.bucket_pack(ts, buf, offs, scale)
        return buf

    def unpack_grads_to_params(self, bk: FlatBucket):
        """Write the (reduced) flat grads back into p.grad (for non-madnn optimizers)."""
        gs = []
        for p in bk.params:
            if p.grad is None or p.grad.stride() != p.stride():
                p.grad = torch.empty_like(p)
            gs.append(p.grad)
        ops.bucket_unpack(gs, bk.grad, bk.offsets, 1.0)

    # ----------------------------------------------------------------- params
    def sync_model_from_master(self, bk: Optional[FlatBucket] = None):
        for b in ([bk] if bk is not None else self.buckets):
            if b.has_master_copy:
                ops.flat_scale_cast(b.master, b.model, 1.0)

    def sync_master_from_model(self, bk: Optional[FlatBucket] = None):
        for b in ([bk] if bk is not None else self.buckets):
            if b.has_master_copy:
                ops.flat_scale_cast(b.model, b.master, 1.0)

    def master_view(self, p: nn.Parameter) -> torch.Tensor:
        """fp32 master value of ``p`` with p's logical shape."""
        bk, off, cl = self.param_info[id(p)]
        return _phys_view(bk.master[off:off + p.numel()], p.shape, cl)

    def params(self) -> List[nn.Parameter]:
        return [p for bk in self.buckets for p in bk.params]

    def numel(self) -> int:
        return sum(p.numel() for p in self.params())

    def bytes(self) -> int:
        tot = 0
        for bk in self.buckets:
            tot += bk.model.numel() * bk.model.element_size()
            if bk.has_master_copy:
                tot += bk.master.numel() * 4
            if bk.grad is not None:
                tot += bk.grad.numel() * bk.grad.element_size()
        return tot
