"""Fused optimizers over flat buckets (K1 FusedSGD, K2 FusedAdam/AdamW).

Reference: Torch7's ``accUpdateGradParameters`` — the gradient step fused into
the weight update, run once per sample by the patched trainer
(datamodule.lua:142).  Here one kernel launch per bucket reads the
flat gradient (already averaged by the DP reducer, or packed locally), updates
the fp32 master and optimizer state, and writes the bf16 model copy the next
forward reads.

The classes subclass ``torch.optim.Optimizer`` so LR schedulers, param groups
and ``state_dict()`` work as usual; the state dict is emitted in per-parameter
form (``momentum_buffer`` / ``exp_avg`` / ``exp_avg_sq``), i.e. the same shape
as ``torch.optim.SGD``/``AdamW`` state, which keeps checkpoints
strategy-agnostic.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
from torch import nn

from .. import ops
from ..parallel.flat import FlatBucket, FlatParamSpace, _phys_view


class NonFiniteGradients(RuntimeError):
    """Raised by a fused optimizer step with ``nonfinite="raise"`` when a gradient is NaN/Inf."""


class _FlatOptimizer(torch.optim.Optimizer):
    _state_names: tuple = ()

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self.space: Optional[FlatParamSpace] = None
        self.grad_source = None          # engine that provides reduced flat grads (DP reducer)
        self.flat_state: Dict[int, Dict[str, torch.Tensor]] = {}
        self.bucket_steps: Dict[int, int] = {}
        self._dscale: Optional[torch.Tensor] = None
        self._pending_load = None
        self.norm_spec = None              # (groups, skip params) for clipping when no engine provides it
        self.nonfinite = "ignore"          # ignore | skip | raise (set from Config.nonfinite by distribute)
        self.skipped_steps = 0

    # ----------------------------------------------------------------- binding
    def bind(self, space: FlatParamSpace):
        """Adopt a FlatParamSpace built over this optimizer's param groups."""
        self.space = space
        self.flat_state = {}
        for bk in space.buckets:
            self.flat_state[bk.index] = {n: torch.zeros_like(bk.master) for n in self._state_names}
            self.bucket_steps[bk.index] = 0
        if self._pending_load is not None:
            sd, self._pending_load = self._pending_load, None
            self.load_state_dict(sd)

    @torch.no_grad()
    def migrate(self, old: dict):
        """Follow a ``FlatParamSpace.relayout``: move every parameter's optimizer state from its
        old bucket slot (``old[id(p)] = (bucket, offset)``) to its new one."""
        self.migrate_begin()
        for bk in self.space.buckets:
            self.migrate_bucket(bk, old)
        self.migrate_end()

    # streaming form, driven by FlatParamSpace.relayout(on_bucket=..., on_release=...)
    def migrate_begin(self):
        self._old_state, self._old_steps = self.flat_state, self.bucket_steps
        self._old_names = {n for v in self._old_state.values() for n in v}
        self.flat_state, self.bucket_steps = {}, {}

    @torch.no_grad()
    def migrate_bucket(self, bk, old: dict):
        st = {n: torch.zeros_like(bk.master) for n in self._state_names if n in self._old_names}
        steps = 0
        for p, off in zip(bk.params, bk.offsets):
            obk, ooff = old[id(p)]
            steps = max(steps, self._old_steps.get(obk.index, 0))
            for n, t in st.items():
                if n in self._old_state.get(obk.index, {}):
                    t[off:off + p.numel()].copy_(self._old_state[obk.index][n][ooff:ooff + p.numel()])
        self.flat_state[bk.index] = st
        self.bucket_steps[bk.index] = steps

    def migrate_release(self, obk):
        self._old_state.pop(obk.index, None)

    def migrate_end(self):
        del self._old_state, self._old_steps, self._old_names

    def _bind_local(self):
        groups = [g["params"] for g in self.param_groups]
        dev = groups[0][0].device
        space = FlatParamSpace(groups, dtype_of=lambda p: p.dtype, bucket_cap_mb=256.0,
                               reduce_dtype=torch.float32, device=dev)
        self.bind(space)

    def _reduced_by_engine(self) -> bool:
        return self.grad_source is not None and getattr(self.grad_source, "sync", None) == "grads"

    def _grads(self, bk: FlatBucket) -> torch.Tensor:
        if not self._reduced_by_engine():
            return self.space.pack_grads(bk, 1.0)
        return self.space.grad_buffer(bk)

    # -------------------------------------------------------------- clipping
    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """GLOBAL-norm clipping fused into the next step (device-side coefficient, no host sync).

        The squared norm of this rank's flat gradients is summed over the groups the engine
        names (``norm_reduction``): the pipeline group (stages hold disjoint parameters; a
        tied parameter counts on its first owner only) and the tensor-parallel group
        (shards count on every rank, replicated parameters on TP rank 0 only), so every rank
        applies the coefficient torch.nn.utils.clip_grad_norm_ would on the whole model."""
        if self.space is None:
            self._bind_local()
        if self._reduced_by_engine():
            self.grad_source.finalize_grads()
        flats = [self._grads(bk) for bk in self.space.buckets]
        self._grads_cached = flats
        groups, skip = self.norm_spec or ([], [])
        if self.grad_source is not None and hasattr(self.grad_source, "norm_reduction"):
            groups, skip = self.grad_source.norm_reduction()
        if not groups and not skip:
            out = ops.grad_norm(flats, max_norm=max_norm)
            self._dscale = out[1:2]
            return out[0]
        sq = ops.grad_norm(flats, max_norm=0.0)[0:1].double().square()
        for p in skip:
            if id(p) not in self.space.param_info:
                continue  # not optimised by this optimizer: contributes no gradient here
            bk, off, _ = self.space.param_info[id(p)]
            i = self.space.buckets.index(bk)
            sq -= flats[i][off:off + p.numel()].double().square().sum()
        sq = sq.float()
        from .. import comm

        for g in groups:
            comm.all_reduce(sq, "sum", group=g)
        norm = sq.clamp_min(0).sqrt()
        self._dscale = (max_norm / (norm + 1e-6)).clamp(max=1.0)
        return norm[0]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self.space is None:
            self._bind_local()
        late = set()
        gs = self.grad_source
        if self._reduced_by_engine():
            if hasattr(gs, "tied_buckets") and getattr(self, "_grads_cached", None) is None:
                # update every other bucket while the cross-stage tied-gradient sum runs
                gs.finalize_grads(wait_tied=False)
                late = gs.tied_buckets()
            else:
                gs.finalize_grads()
        cached = getattr(self, "_grads_cached", None)
        if self.nonfinite != "ignore":
            finite = self._grads_finite(late, cached)
            cached = getattr(self, "_grads_cached", None)   # packed by the check in local-pack mode
        else:
            finite = True
        if not finite:
            self.skipped_steps += 1
            if self.nonfinite == "raise":
                # nothing of this step survives into the next one: a caller that catches the
                # error, zeroes its gradients and continues must not get these packed NaN flats
                # (or the NaN clip scale) back
                self._grads_cached = None
                self._dscale = None
                raise NonFiniteGradients(f"non-finite gradients at optimizer step {self.skipped_steps}")
            from ..utils.logging import get_logger

            get_logger().warning("madnn: non-finite gradients; optimizer step skipped (%d so far)", self.skipped_steps)
            if late:
                gs.finalize_grads()
            for bk in self.space.buckets:  # nothing of this step's gradients may leak into the next
                if bk.grad is not None:
                    bk.grad.zero_()
            self._grads_cached = None
            self._dscale = None
            if self.grad_source is not None:
                self.grad_source.after_step()
            return loss
        order = [i for i, bk in enumerate(self.space.buckets) if bk.index not in late] + \
                [i for i, bk in enumerate(self.space.buckets) if bk.index in late]
        for i in order:
            bk = self.space.buckets[i]
            if late and bk.index in late:
                gs.finalize_grads()
                late = set()
            g = cached[i] if cached is not None else self._grads(bk)
            group = self.param_groups[bk.group_id]
            self.bucket_steps[bk.index] += 1
            self._update(bk, g, group, self.flat_state[bk.index], self.bucket_steps[bk.index])
        self._grads_cached = None
        self._dscale = None
        if self.grad_source is not None:
            self.grad_source.after_step()
        return loss

    @torch.no_grad()
    def _grads_finite(self, late, cached) -> bool:
        """Whether every reduced gradient of the step is finite -- on EVERY rank (one MAX
        all-reduce of a flag over the world group, so pipeline stages holding different
        parameters skip or step together).  One host sync per step: only with ``nonfinite`` on."""
        if late:
            self.grad_source.finalize_grads()
        flats = cached if cached is not None else [self._grads(bk) for bk in self.space.buckets]
        if cached is None:
            self._grads_cached = flats
        sq = ops.grad_norm(flats, max_norm=0.0)[0:1].float()
        bad = (~torch.isfinite(sq)).float()
        from .. import comm
        import torch.distributed as dist

        if dist.is_initialized() and dist.get_world_size() > 1:
            comm.all_reduce(bad, "max")
        return float(bad.item()) == 0.0

    def zero_grad(self, set_to_none: bool = True):
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is not None:
                    if set_to_none:
                        p.grad = None
                    else:
                        p.grad.zero_()

    def _model_out(self, bk: FlatBucket):
        return bk.model if bk.has_master_copy else None

    def _update(self, bk, grad, group, st, step):  # pragma: no cover - abstract
        raise NotImplementedError

    # ------------------------------------------------------------ state dict
    def _param_index(self):
        idx, k = {}, 0
        for g in self.param_groups:
            for p in g["params"]:
                idx[id(p)] = k
                k += 1
        return idx

    def state_dict(self):
        groups = []
        k = 0
        for g in self.param_groups:
            d = {key: v for key, v in g.items() if key != "params"}
            d["params"] = list(range(k, k + len(g["params"])))
            k += len(g["params"])
            groups.append(d)
        state = {}
        if self.space is not None:
            idx = self._param_index()
            for bk in self.space.buckets:
                st = self.flat_state[bk.index]
                for p, off in zip(bk.params, bk.offsets):
                    cl = self.space.param_info[id(p)][2]
                    entry = {n: _phys_view(st[n][off:off + p.numel()], p.shape, cl).clone() for n in st}
                    entry["step"] = torch.tensor(float(self.bucket_steps[bk.index]))
                    state[idx[id(p)]] = self._export_names(entry)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        for g, sg in zip(self.param_groups, sd["param_groups"]):
            for key, v in sg.items():
                if key != "params":
                    g[key] = v
        if self.space is None:
            # the flat state needs the space; hyper-parameters are applied NOW (a later
            # g["lr"] = ... must not be undone when the space binds at the first step)
            self._pending_load = {"state": sd["state"], "param_groups": []}
            return
        idx = self._param_index()
        for bk in self.space.buckets:
            st = self.flat_state[bk.index]
            for p, off in zip(bk.params, bk.offsets):
                e = sd["state"].get(idx[id(p)]) or sd["state"].get(str(idx[id(p)]))
                if e is None:
                    continue
                e = self._import_names(e)
                cl = self.space.param_info[id(p)][2]
                for n in st:
                    if n in e:
                        _phys_view(st[n][off:off + p.numel()], p.shape, cl).copy_(e[n])
                if "step" in e:
                    self.bucket_steps[bk.index] = int(float(e["step"]))

    def _export_names(self, e):
        return e

    def _import_names(self, e):
        return e


class FusedSGD(_FlatOptimizer):
    """SGD with momentum / dampening / nesterov / weight decay (torch.optim.SGD semantics)."""

    _state_names = ("momentum",)

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))

    def bind(self, space):
        super().bind(space)
        if all(g["momentum"] == 0 for g in self.param_groups):
            for st in self.flat_state.values():
                st.pop("momentum", None)

    def _update(self, bk, grad, group, st, step):
        ops.sgd_step(bk.master, grad, st.get("momentum"), self._model_out(bk), lr=group["lr"],
                     momentum=group["momentum"], dampening=group["dampening"],
                     weight_decay=group["weight_decay"], nesterov=group["nesterov"], first_step=(step == 1),
                     grad_scale=1.0, dscale=self._dscale)

    def _export_names(self, e):
        if "momentum" in e:
            e["momentum_buffer"] = e.pop("momentum")
        return e

    def _import_names(self, e):
        e = dict(e)
        if "momentum_buffer" in e:
            e["momentum"] = e.pop("momentum_buffer")
        return e


class FusedAdam(_FlatOptimizer):
    """Adam / AdamW (decoupled weight decay when ``adamw=True``), torch semantics."""

    _state_names = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 adamw: bool = True):
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, adamw=adamw))

    def _update(self, bk, grad, group, st, step):
        b1, b2 = group["betas"]
        ops.adam_step(bk.master, grad, st["exp_avg"], st["exp_avg_sq"], self._model_out(bk), lr=group["lr"],
                      beta1=b1, beta2=b2, eps=group["eps"], weight_decay=group["weight_decay"],
                      adamw=group["adamw"], step=step, grad_scale=1.0, dscale=self._dscale)


def FusedAdamW(params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2):
    return FusedAdam(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, adamw=True)


__all__ = ["FusedSGD", "FusedAdam", "FusedAdamW", "NonFiniteGradients"]
