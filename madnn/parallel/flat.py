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
* each bucket owns a ``grad`` buffer that RCCL reduces in place.  By default
  (``reduce_dtype=None``) it has the bucket's own dtype -- bf16 for bf16
  parameters (half the all-reduce bytes of fp32; the fp32 master update is
  unchanged), fp32 for fp32 norm parameters;
* gradients land in that buffer one of two ways: the layers that own their
  backward (``ops.linear``: every zoo transformer Linear) write the weight
  gradient STRAIGHT into the parameter's slot (:meth:`FlatParamSpace.grad_sink`;
  autograd adopts the view as ``p.grad``, no copy), everything else is copied
  in by the K4 pack kernel when its bucket is ready;
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
        self.grad_dtype: Optional[torch.dtype] = None

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
                 reduce_dtype: Optional[torch.dtype] = None,
                 channels_last_of: Optional[Callable[[nn.Parameter], bool]] = None,
                 device: Optional[torch.device] = None,
                 order: Optional[Sequence[int]] = None):
        self.reduce_dtype = reduce_dtype        # None: every bucket reduces in its own dtype
        self.bucket_cap_mb = bucket_cap_mb
        self.buckets: List[FlatBucket] = []
        self.param_info: Dict[int, tuple] = {}  # id(p) -> (bucket, offset, channels_last)
        self.group_of_param: Dict[int, int] = {}
        self._sinks_on = False
        self._groups = [list(g) for g in param_groups]
        self._dtype_of = dtype_of
        self._cl_of = channels_last_of or (lambda p: False)
        self._device = device
        self._layout(param_groups, dtype_of, order)
        for bk in self.buckets:
            self._materialize(bk, device, self._cl_of)

    # ------------------------------------------------------------ re-layout
    def layout_is_contiguous(self, observed: Sequence[int]) -> bool:
        """True when every bucket's parameters arrive as one contiguous run of the observed
        gradient order -- each bucket is ready as soon as its own gradients are, never held
        back by a parameter that backward reaches much later."""
        where = {id(p): bk.index for bk in self.buckets for p in bk.params}
        seq = [where[i] for i in observed if i in where]
        runs = [b for k, b in enumerate(seq) if k == 0 or b != seq[k - 1]]
        return len(runs) == len(set(runs))

    @torch.no_grad()
    def relayout(self, observed: Sequence[int], on_bucket=None, on_release=None):
        """Re-lay the buckets in the OBSERVED gradient-ready order: values move
        exactly (fp32 masters copied, compute copies re-derived), parameters are re-pointed at
        the new buffers.  Returns ``{id(p): (old bucket, old offset)}`` for state migration.

        Streaming: ``on_bucket(new_bucket, old)`` runs right after each new bucket is built (the
        optimizer moves that bucket's state then), and an old bucket's buffers are dropped --
        ``on_release(old_bucket)`` lets the optimizer drop its state -- as soon as every one of
        its parameters has moved.  The transient is a few buckets, not a second copy of every
        master / moment buffer (Llama-3 8B on one GPU: +96 GB without streaming)."""
        old = {id(p): (bk, off) for bk in self.buckets for p, off in zip(bk.params, bk.offsets)}
        left = {bk.index: len(bk.params) for bk in self.buckets}
        old_info = dict(self.param_info)
        sinks = self._sinks_on
        if sinks:
            self.disable_grad_sinks()
        self.buckets, self.param_info, self.group_of_param = [], {}, {}
        self._layout(self._groups, self._dtype_of, observed)
        for bk in self.buckets:
            dev = old[id(bk.params[0])][0].master.device
            master = torch.zeros(bk.numel, dtype=torch.float32, device=dev)
            model = master if bk.dtype == torch.float32 else torch.empty(bk.numel, dtype=bk.dtype, device=dev)
            for p, off in zip(bk.params, bk.offsets):
                obk, ooff = old[id(p)]
                cl = old_info[id(p)][2]
                n = p.numel()
                master[off:off + n].copy_(obk.master[ooff:ooff + n])
                if model is not master:
                    model[off:off + n].copy_(obk.model[ooff:ooff + n])
                self.param_info[id(p)] = (bk, off, cl)
                p.data = _phys_view(model[off:off + n], p.shape, cl)
                p._madnn_home = self
            bk.master, bk.model = master, model
            if on_bucket is not None:
                on_bucket(bk, old)
            for p in bk.params:
                obk = old[id(p)][0]
                left[obk.index] -= 1
                if left[obk.index] == 0:  # every parameter of obk has moved: free its buffers now
                    if on_release is not None:
                        on_release(obk)
                    obk.master = obk.model = obk.grad = None
        if sinks:
            self.enable_grad_sinks()
        return old

    def _layout(self, param_groups, dtype_of, order=None):
        """Assign parameters to buckets.  ``order``: ids of parameters in OBSERVED gradient-ready
        order (from a profiled backward); default: reverse registration order, which is what
        backward roughly follows."""
        rank = {pid: i for i, pid in enumerate(order)} if order else None
        for gi, group in enumerate(param_groups):
            plist = [p for p in group if p.requires_grad]
            if rank is None:
                plist = list(reversed(plist))
            else:
                n = len(rank)
                plist = sorted(plist, key=lambda p: rank.get(id(p), n))
            by_dtype: Dict[torch.dtype, List[nn.Parameter]] = {}
            for p in plist:
                by_dtype.setdefault(dtype_of(p), []).append(p)
            for dt, ps in by_dtype.items():
                gdt = self.reduce_dtype or dt
                cap_elems = int(self.bucket_cap_mb * 1024 * 1024 / torch.tensor([], dtype=gdt).element_size())
                bucket_of, offset_of, sizes = native_runtime.plan_buckets([p.numel() for p in ps], cap_elems, ALIGN)
                base = len(self.buckets)
                for k in range(len(sizes)):
                    bk = FlatBucket(base + k, dt, gi)
                    bk.grad_dtype = gdt
                    self.buckets.append(bk)
                for p, b, off in zip(ps, bucket_of, offset_of):
                    bk = self.buckets[base + b]
                    bk.params.append(p)
                    bk.offsets.append(off)
                    self.group_of_param[id(p)] = gi
                for k, sz in enumerate(sizes):
                    self.buckets[base + k].numel = int(sz)

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
            p._madnn_home = self  # the space whose fp32 master is this parameter's true value
            # an existing p.grad stays valid: pack_grads re-layouts it if its strides differ
        bk.model = model
        bk.master = master

    # ------------------------------------------------------------------ grads
    def grad_buffer(self, bk: FlatBucket) -> torch.Tensor:
        if bk.grad is None:
            bk.grad = torch.zeros(bk.numel, dtype=bk.grad_dtype or self.reduce_dtype or torch.float32,
                                  device=bk.model.device)
        return bk.grad

    # ------------------------------------------------------- direct-write sinks
    def enable_grad_sinks(self) -> int:
        """Let layers that own their backward write weight gradients straight into the
        buckets: every parameter whose bucket reduces in its own dtype gets a sink (see
        :func:`madnn.ops.grad_sink`).  Returns the number of parameters with a sink."""
        n = 0
        for bk in self.buckets:
            if bk.grad_dtype != bk.dtype:
                continue
            self.grad_buffer(bk)
            for p in bk.params:
                p._madnn_space = self
                n += 1
        self._sinks_on = n > 0
        return n

    def disable_grad_sinks(self) -> None:
        for bk in self.buckets:
            for p in bk.params:
                if getattr(p, "_madnn_space", None) is self:
                    del p._madnn_space
        self._sinks_on = False

    def grad_slot(self, p: nn.Parameter) -> Optional[torch.Tensor]:
        """A FRESH view of ``p``'s slot in its bucket's gradient buffer (same shape and strides
        as ``p``), or None when ``p``'s bucket reduces in another dtype.  Fresh, so autograd's
        AccumulateGrad can adopt it as ``p.grad`` without a copy."""
        bk, off, cl = self.param_info[id(p)]
        if bk.grad_dtype != bk.dtype:
            return None
        return _phys_view(self.grad_buffer(bk)[off:off + p.numel()], p.shape, cl)

    def _in_place(self, p, bk, off) -> bool:
        g = p.grad
        return g is not None and g.data_ptr() == bk.grad.data_ptr() + off * bk.grad.element_size() \
            and g.dtype == bk.grad.dtype

    def bucket_grads(self, bk: FlatBucket):
        """(tensors, offsets) of the params of ``bk`` that hold a grad NOT already in the bucket,
        and the offsets/sizes of the params without any grad."""
        ts, offs, missing = [], [], []
        buf = self.grad_buffer(bk)
        for p, off in zip(bk.params, bk.offsets):
            g = p.grad
            if g is None:
                missing.append((off, p.numel()))
                continue
            if self._in_place(p, bk, off):
                continue
            if g.stride() != p.stride() or not is_dense(g):
                g = torch.empty_like(p).copy_(g)  # match the bucket's physical layout
            ts.append(g)
            offs.append(off)
        return ts, offs, missing

    def pack_grads(self, bk: FlatBucket, scale: float = 1.0) -> torch.Tensor:
        """Gather ``bk``'s gradients into its flat buffer (x ``scale``).  Gradients already
        written in place are left alone -- callers that need a scale on those too must pass
        scale 1.0 and scale in the reduction (RCCL's in-kernel average)."""
        buf = self.grad_buffer(bk)
        ts, offs, missing = self.bucket_grads(bk)
        for off, n in missing:
            buf[off:off + n].zero_()  # params without grad contribute zeros (unused in this step)
        ops.bucket_pack(ts, buf, offs, scale)
        if scale != 1.0 and len(ts) + len(missing) < len(bk.params):
            raise RuntimeError("pack_grads: in-place gradients cannot take a pack scale")
        return buf

    def packed_fraction(self, bk: FlatBucket) -> float:
        """Fraction of ``bk``'s elements whose gradient needed a copy (diagnostics)."""
        tot = sum(p.numel() for p in bk.params) or 1
        return sum(p.numel() for p, off in zip(bk.params, bk.offsets) if p.grad is not None
                   and not self._in_place(p, bk, off)) / tot

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
