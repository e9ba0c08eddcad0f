"""Data-parallel engine: bucketed, backward-overlapped gradient averaging over
RCCL, plus the reference's periodic parameter averaging (local SGD).

Reference behaviour:
* ``synchronizeModel`` (datamodule.lua:211-224) all-reduces and averages every
  parameter and gradient tensor, one blocking collective per tensor, after
  backward, every K samples (the "batchSize" period, datamodule.lua:102,151);
* that hook is installed by globally monkey-patching ``nn.Sequential:backward``
  and ``nn.StochasticGradient:train`` (datamodule.lua:83,117).

MI355X-native redesign:
* hooks are installed on the wrapped root's parameters only
  (``register_post_accumulate_grad_hook``) — no global patching (SURVEY A-8);
* gradients are averaged in flat buckets: as soon as the last gradient of a
  bucket is accumulated, the K4 pack kernel (1/W fused) runs on a dedicated
  high-priority HIP stream and the bucket's RCCL all-reduce is issued
  asynchronously, so communication overlaps the rest of backward;
* the fused optimizer consumes the reduced flat buffers directly;
* ``sync="params"`` keeps the reference's period-K model averaging (A-3),
  ``sync="manual"`` mirrors ``batchSize = -1`` (datamodule.lua:45).
"""
from __future__ import annotations

import contextlib
import math
import time
from typing import Optional, Union

import torch
from torch import nn

from .. import comm
from .. import runtime as rt
from ..utils.logging import get_logger
from .flat import FlatBucket, FlatParamSpace


def default_sync_period(local_size: int) -> int:
    """Reference sync-period heuristic (datamodule.lua:68-78): 1/10/50/100 samples."""
    if local_size < 1000:
        return 1
    if local_size < 2500:
        return 10
    if local_size < 5000:
        return 50
    return 100


def auto_sync_period(step_s: float, sync_s: float, budget: float = 0.05, k_max: int = 10000) -> int:
    """Smallest K with ``sync_s <= budget * K * step_s`` (1 <= K <= k_max)."""
    if step_s <= 0:
        return k_max if sync_s > 0 else 1
    return int(min(max(math.ceil(sync_s / (budget * step_s) - 1e-9), 1), k_max))


def robustness_tick(step: int, group=None) -> None:
    """Per-optimizer-step robustness hooks shared by every engine and the Trainer:

    * ``MADNN_FAULT=rank:step:kind`` fault injection (``utils.fault``), used by the tests that
      prove a hung or crashed rank becomes a process-group timeout and a launcher teardown;
    * the K5 one-shot all-reduce's error word (a timed-out peer wait raises, never trains on);
    * with ``check_collectives`` on (``Config.check_collectives`` / ``MADNN_CHECK_COLLECTIVES=1``),
      every ``MADNN_CHECK_EVERY`` (default 50) steps all ranks compare the running fingerprint
      of their collective sequence and raise on divergence."""
    from ..utils.fault import maybe_fail

    maybe_fail(step)
    from ..comm import oneshot

    if oneshot._registry:
        oneshot.poll_all()   # a K5 call whose peer wait timed out raises here
    if comm.order_check_enabled():
        every = comm.check_every()
        if every > 0 and step % every == 0:
            comm.verify_order(group)


def _cast_inputs(obj, dtype, channels_last):
    if isinstance(obj, torch.Tensor):
        if obj.is_floating_point() and dtype is not None and obj.dtype != dtype:
            obj = obj.to(dtype)
        if channels_last and obj.dim() == 4 and obj.is_floating_point():
            obj = obj.contiguous(memory_format=torch.channels_last)
        return obj
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cast_inputs(o, dtype, channels_last) for o in obj)
    if isinstance(obj, dict):
        return {k: _cast_inputs(v, dtype, channels_last) for k, v in obj.items()}
    return obj


def _leading_dim(args, kwargs) -> int:
    """Samples in one forward's input: the leading dim of its first tensor (0 if none)."""
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor):
            return int(a.shape[0]) if a.dim() > 0 else 1
        if isinstance(a, (list, tuple)) and a and isinstance(a[0], torch.Tensor):
            return int(a[0].shape[0]) if a[0].dim() > 0 else 1
        if isinstance(a, dict):
            n = _leading_dim((), a)
            if n:
                return n
    return 0


class DataParallel(nn.Module):
    """Wraps a module whose parameters live in a :class:`FlatParamSpace`."""

    def __init__(self, module: nn.Module, space: FlatParamSpace, *, group=None, src_rank: int = 0,
                 sync: str = "grads", sync_every: Union[int, str] = 1, overlap: bool = True,
                 cast_dtype: Optional[torch.dtype] = None, channels_last: bool = False,
                 unpack_grads: bool = False, broadcast_buffers: bool = True, find_unused: bool = True,
                 sync_comm: bool = False, grad_sinks: bool = True, rebuild_buckets: bool = True,
                 sync_samples: Optional[int] = None, sync_budget: float = 0.05):
        super().__init__()
        self.module = module
        self.space = space
        self.group = group
        self.src_rank = src_rank
        self.world = rt.get_world_size(group)
        self.sync = sync
        # sync="params" period: every ``sync_every`` optimizer steps, or "auto" (measured, see
        # _auto_period), or -- ``sync_samples`` -- whenever the count of trained SAMPLES crosses a
        # multiple of it (the reference's unit, datamodule.lua:102,151)
        self.sync_every = "auto" if sync_every == "auto" else max(int(sync_every), 1)
        self.sync_samples = int(sync_samples) if sync_samples else None
        self.sync_budget = float(sync_budget)
        self.sync_calibration = None          # sync_every="auto": the measurement and the chosen K
        self._samples = 0
        self._fwd_samples = 0
        self._per_step = None                 # agreed samples per step (sync_samples; _params_tick)
        self._calib = None
        self._period_origin = 0
        self.cast_dtype = cast_dtype
        self.channels_last = channels_last
        self.unpack_grads = unpack_grads
        self.find_unused = find_unused
        dev = space.buckets[0].model.device if space.buckets else torch.device("cpu")
        self.is_cuda = dev.type == "cuda"
        self.comm_stream = None
        if self.is_cuda and overlap and not sync_comm:
            # high priority so the pack + RCCL enqueue is not starved by backward kernels
            self.comm_stream = torch.cuda.Stream(device=dev, priority=-1)
        self._sync_enabled = True
        self.defer_flush = False
        self._in_backward = False
        self._needs_finalize = False
        self._steps = 0
        self._backwards = 0
        self._hooks = []
        self.stats = {"buckets_launched": 0, "bytes_reduced": 0}
        # per-step comm observability (HIP events; read one step later, never synchronising):
        # exposed = compute-stream time from the end of backward to the reduced gradients
        self._ev = {}
        self._last_ev = None
        self._step_bytes = 0
        self.broadcast_state(broadcast_buffers)
        self.grad_sinks = 0
        self.optimizer = None                 # fused optimizer bound to ``space`` (set by distribute)
        self.rebuild_buckets = rebuild_buckets
        self._observe = [] if (sync == "grads" and rebuild_buckets) else None
        self.rebuilt = False
        if sync == "grads":
            self._install_hooks()
            if not unpack_grads and grad_sinks:
                # fused optimizer reads the buckets: layers may write weight grads straight in
                self.grad_sinks = space.enable_grad_sinks()

    # ---------------------------------------------------------------- setup
    @torch.no_grad()
    def broadcast_state(self, buffers: bool = True):
        """Identical start on every replica (fixes SURVEY A-6: always broadcast).  Issued
        whenever a process group exists -- also at world size 1 under a launcher, so the
        RCCL broadcast path is the one the 1-GPU rehearsal exercises."""
        if comm._local(self.group):
            return
        for bk in self.space.buckets:
            comm.broadcast(bk.master, src=self.src_rank, group=self.group)
        self.space.sync_model_from_master()
        if buffers:
            for b in self.module.buffers():
                if b.is_floating_point() or b.dtype in (torch.int64, torch.long):
                    comm.broadcast(b, src=self.src_rank, group=self.group)

    def _install_hooks(self):
        self._next_launch = 0
        for bk in self.space.buckets:
            bk.pending = len(bk.params)
            for p in bk.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(bk)))

    def _make_hook(self, bk: FlatBucket):
        def hook(_p):
            if not self._sync_enabled:
                return
            if self._observe is not None:
                self._observe.append(id(_p))
            if not self._in_backward:
                self._in_backward = True
                if self._needs_finalize:
                    # a second backward before the optimizer consumed the first one's reduced
                    # gradients (plain accumulation without no_sync): p.grad now holds the local
                    # SUM of both, so re-pack and re-reduce every bucket (torch DDP semantics:
                    # each backward reduces).  forward() already ordered this backward's in-place
                    # accumulation after the first reduction's packs.
                    self._rearm()
                torch.autograd.Variable._execution_engine.queue_callback(self._on_backward_end)
            bk.pending -= 1
            if bk.pending == 0:
                self._launch_ready()

        return hook

    def _launch_ready(self):
        """Launch every ready bucket in INDEX order (torch DDP's rule): collectives on one
        communicator must be issued in the same order on every rank, and replicas whose
        gradients become ready in different orders (data-dependent branches, parameters unused
        on one rank) would otherwise issue their bucket all-reduces in different orders."""
        bks = self.space.buckets
        while self._next_launch < len(bks):
            bk = bks[self._next_launch]
            if bk.pending > 0 and not bk.launched:
                return
            if not bk.launched:
                self._launch(bk)
            self._next_launch += 1

    # ------------------------------------------------------------ reduction
    def _launch(self, bk: FlatBucket):
        # pack with no scale: gradients written in place by their layers (grad sinks) cannot take
        # one, so the 1/W average rides in RCCL's in-kernel AVG reduction (a plain sum at W = 1)
        scale, op = 1.0, ("avg" if self.world > 1 else "sum")
        if self.comm_stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(bk.model.device))
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                if "comm_start" not in self._ev and self._timing():
                    self._ev["comm_start"] = torch.cuda.Event(enable_timing=True)
                    self._ev["comm_start"].record(self.comm_stream)
                for p in bk.params:
                    if p.grad is not None:
                        p.grad.record_stream(self.comm_stream)
                buf = self.space.pack_grads(bk, scale)
                self._maybe_corrupt(buf)
                bk.work = comm.all_reduce(buf, op, group=self.group, async_op=True)
        else:
            buf = self.space.pack_grads(bk, scale)
            self._maybe_corrupt(buf)
            bk.work = comm.all_reduce(buf, op, group=self.group, async_op=True)
        bk.launched = True
        self.stats["buckets_launched"] += 1
        self.stats["bytes_reduced"] += buf.numel() * buf.element_size()
        self._step_bytes += buf.numel() * buf.element_size()

    def _maybe_corrupt(self, buf):
        import os

        if os.environ.get("MADNN_FAULT"):
            from ..utils.fault import maybe_corrupt

            maybe_corrupt(self._steps + 1, buf)  # fault injection: NaN gradients of this step

    def _on_backward_end(self):
        self._in_backward = False
        self._backwards += 1
        if not self.defer_flush:
            self.flush()

    def flush(self):
        """End of the gradient-producing backward(s): launch the buckets whose parameters got
        no gradient and mark the step for finalisation.  Runs from the autograd end callback,
        or -- with ``defer_flush`` (the pipeline engine, whose chunks finish their last
        microbatch at different times) -- explicitly after the LAST backward."""
        if self._timing():
            self._ev["bwd_end"] = torch.cuda.Event(enable_timing=True)
            self._ev["bwd_end"].record()
        for bk in self.space.buckets:
            if not bk.launched:
                if bk.pending > 0 and not self.find_unused:
                    raise RuntimeError(f"bucket {bk.index} had parameters without gradients; "
                                       "set find_unused=True")
                self._launch(bk)
        self._next_launch = len(self.space.buckets)
        self._needs_finalize = True

    def _wait_works(self, record_end: bool = False):
        """The current stream waits for every outstanding bucket reduction; buckets re-armed."""
        cur = torch.cuda.current_stream() if self.is_cuda else None
        if self.comm_stream is not None:
            with torch.cuda.stream(self.comm_stream):
                for bk in self.space.buckets:
                    if bk.work is not None:
                        bk.work.wait()  # comm stream waits for the collective
                        bk.work = None
                if record_end and "comm_start" in self._ev and self._timing():
                    self._ev["comm_end"] = torch.cuda.Event(enable_timing=True)
                    self._ev["comm_end"].record(self.comm_stream)
            cur.wait_stream(self.comm_stream)
        for bk in self.space.buckets:
            if bk.work is not None:
                bk.work.wait()
                bk.work = None
            bk.launched = False
            bk.pending = len(bk.params)
        self._next_launch = 0
        return cur

    def _rearm(self):
        self._wait_works()
        self._needs_finalize = False
        self.stats["rearmed"] = self.stats.get("rearmed", 0) + 1

    def finalize_grads(self):
        """Make the current stream wait for every bucket's reduction (idempotent)."""
        if not self._needs_finalize:
            return
        cur = self._wait_works(record_end=True)
        if self._timing() and "bwd_end" in self._ev:
            self._ev["final"] = torch.cuda.Event(enable_timing=True)
            self._ev["final"].record(cur)
        self._last_ev, self._ev = (self._ev, self._step_bytes), {}
        self._step_bytes = 0
        for bk in self.space.buckets:
            if self.unpack_grads:
                self.space.unpack_grads_to_params(bk)
            else:
                for p in bk.params:
                    p.grad = None
        self._needs_finalize = False

    def _timing(self) -> bool:
        """Per-step timing events (comm_metrics) -- not while the step is captured in a graph."""
        from ..utils.graphs import capturing

        return self.is_cuda and not capturing()

    def comm_metrics(self) -> dict:
        """Comm numbers of the last finalized step (blocks on that step's events only):
        ``comm_exposed_ms`` (compute stream stalled after backward waiting for reduced grads),
        ``comm_ms`` (first bucket launch -> last reduction done, overlapped with backward),
        ``allreduce_bytes`` and ``busbw_gbps`` (ring bus bandwidth over ``comm_ms``)."""
        if self._last_ev is None:
            return {}
        ev, nbytes = self._last_ev
        out = {"allreduce_bytes": nbytes}
        if "bwd_end" in ev and "final" in ev:
            ev["final"].synchronize()
            out["comm_exposed_ms"] = max(ev["bwd_end"].elapsed_time(ev["final"]), 0.0)
        if "comm_start" in ev and "comm_end" in ev:
            ev["comm_end"].synchronize()
            ms = ev["comm_start"].elapsed_time(ev["comm_end"])
            out["comm_ms"] = ms
            if ms > 0 and self.world > 1:
                out["busbw_gbps"] = 2.0 * (self.world - 1) / self.world * nbytes / (ms * 1e-3) / 1e9
        return out

    def norm_reduction(self):
        """Gradient-norm reduction spec for clipping: replicas hold identical reduced gradients
        (nothing to sum); a tensor-parallel inner layout sets ``_norm_spec``."""
        return getattr(self, "_norm_spec", ([], []))

    def after_step(self):
        """Called by the fused optimizer after each step: the sync="params" period, then the
        robustness hooks (fault injection, collective-order check)."""
        self._steps += 1
        if self._steps == 1 and self.world > 1 and not comm._local(self.group):
            # shapes missing from the shipped tuning table were timed on each replica on its own:
            # adopt the source rank's choices so every replica runs the same kernels from now on
            from .. import ops

            ops.sync_choices(self.group, src=self.src_rank)
        if self._observe is not None:
            self._maybe_relayout()
        if self.sync == "params":
            self._params_tick()
        robustness_tick(self._steps, self.group)

    # -------------------------------------------------------- sync period
    def _params_tick(self):
        n, self._fwd_samples = self._fwd_samples, 0
        if self.sync_samples is not None:
            # the averaging is a collective: every replica must reach it at the same step.  The
            # samples a step counts are agreed once (MIN over the group at the first step) and
            # the counter then advances by that amount on every rank, so the decision is a
            # function of the step count alone -- a rank with a larger shard or a short last
            # batch cannot drift off its peers
            if self._per_step is None:
                self._per_step = self._agree_min(max(n, 1))
            before = self._samples
            self._samples += self._per_step
            if self._samples // self.sync_samples > before // self.sync_samples:
                self.average_parameters()
        elif self.sync_every == "auto":
            self._auto_period()
        elif (self._steps - self._period_origin) % self.sync_every == 0:
            self.average_parameters()

    def _agree_min(self, v: int) -> int:
        if comm._local(self.group) or self.world <= 1:
            return int(v)
        dev = self.space.buckets[0].master.device if self.space.buckets else torch.device("cpu")
        t = torch.tensor([-int(v)], dtype=torch.float64, device=dev)
        comm.all_reduce(t, "max", group=self.group)
        return int(-t.item())

    AUTO_WARMUP = 1   # steps averaged every step before timing starts (allocator, kernel choices)
    AUTO_MEASURE = 3  # steps timed: compute since the previous average ended, then the average

    def _clock(self) -> float:
        if self.is_cuda:
            torch.cuda.synchronize()
        return time.perf_counter()

    def _auto_period(self):
        """sync_every="auto": the reference's intended period from measured communication speed
        (``comm_speed`` -> ``optimize_sync``, datamodule.lua:40-47,65-78,280-303), done on the job.
        The first AUTO_WARMUP + AUTO_MEASURE steps average every step (K = 1 is always correct);
        the measured ones time the compute since the previous average and the average itself.
        Every rank then takes the MAX of both over the group and picks the smallest K with
        ``sync <= sync_budget * K * step``, so all replicas agree on K.  The device synchronises
        only during these few steps."""
        c = self._calib
        if c is None:
            c = self._calib = {"step": [], "sync": [], "t_end": None}
        k = self._steps
        now = self._clock()
        if c["t_end"] is not None and k > self.AUTO_WARMUP:
            c["step"].append(now - c["t_end"])
            t0 = now
            self.average_parameters()
            now = self._clock()
            c["sync"].append(now - t0)
        else:
            self.average_parameters()
            now = self._clock()
        c["t_end"] = now
        if len(c["sync"]) < self.AUTO_MEASURE:
            return
        step_s = sum(c["step"]) / len(c["step"])
        sync_s = sum(c["sync"]) / len(c["sync"])
        t = torch.tensor([step_s, sync_s], dtype=torch.float64,
                         device=self.space.buckets[0].master.device if self.space.buckets else "cpu")
        if not comm._local(self.group):
            comm.all_reduce(t, "max", group=self.group)
        step_s, sync_s = float(t[0]), float(t[1])
        kk = auto_sync_period(step_s, sync_s, self.sync_budget)
        self.sync_every = kk
        self._period_origin = k
        self._calib = None
        self.sync_calibration = {"step_ms": step_s * 1e3, "sync_ms": sync_s * 1e3, "budget": self.sync_budget,
                                 "K": kk, "decided_at_step": k}
        get_logger().info("madnn dp: sync period auto -> K=%d steps (step %.2f ms, parameter average %.2f ms, "
                          "budget %.0f%%)", kk, step_s * 1e3, sync_s * 1e3, 100 * self.sync_budget)

    def _maybe_relayout(self):
        """After the first step: if the buckets did not fill in the order backward produced
        gradients, re-lay them in the observed order (the source rank's observation, broadcast
        by :meth:`_agree_on_order`, so layouts stay identical across replicas)."""
        seen = self._agree_on_order(self._observe)
        self._observe = None
        if not seen or self.space.layout_is_contiguous(seen):
            return
        if self.optimizer is None and self.unpack_grads is False:
            return  # a flat state we cannot migrate
        opt = self.optimizer
        if opt is not None:
            opt.migrate_begin()
            self.space.relayout(seen, on_bucket=opt.migrate_bucket, on_release=opt.migrate_release)
            opt.migrate_end()
        else:
            self.space.relayout(seen)
        for h in self._hooks:
            h.remove()
        self._hooks.clear()
        self._install_hooks()
        self.rebuilt = True
        get_logger().info("madnn dp: re-laid %d buckets in the observed gradient order", len(self.space.buckets))

    def _agree_on_order(self, seen):
        """The gradient order every replica re-lays its buckets by: this group's source rank's
        observation, broadcast as indices into the (rank-independent) parameter registration
        order.  Ranks may observe different orders (data-dependent branches, parameters unused
        on one rank only); buckets built from different orders would all-reduce unrelated
        slices, so -- as torch DDP does with its rebuilt buckets -- one rank decides."""
        canon = [p for g in self.space._groups for p in g if p.requires_grad]
        if comm._local(self.group) or self.world <= 1:
            return seen
        idx_of = {id(p): i for i, p in enumerate(canon)}
        order, used = [], set()
        for i in seen or ():
            k = idx_of.get(i)
            if k is not None and k not in used:
                used.add(k)
                order.append(k)
        dev = self.space.buckets[0].master.device if self.space.buckets else torch.device("cpu")
        t = torch.full((len(canon),), -1, dtype=torch.int64, device=dev)
        if order:
            t[:len(order)] = torch.tensor(order, dtype=torch.int64, device=dev)
        comm.broadcast(t, src=self.src_rank, group=self.group)
        return [id(canon[k]) for k in t.tolist() if k >= 0]

    @torch.no_grad()
    def average_parameters(self):
        """Reference periodic model averaging (datamodule.lua:214-218), bucketed."""
        if comm._local(self.group):
            return
        for bk in self.space.buckets:
            comm.all_reduce(bk.master, "sum", group=self.group)
            bk.master.mul_(1.0 / self.world)
        self.space.sync_model_from_master()

    def __getattr__(self, name):
        """Attributes the engine does not have resolve on the wrapped module (``eng.h[0]``,
        ``eng.loss_fn`` of a model), so a distributed model reads like the original."""
        try:
            return super().__getattr__(name)
        except AttributeError:
            mods = self.__dict__.get("_modules", {})
            if "module" in mods and name != "module":
                return getattr(mods["module"], name)
            raise

    # -------------------------------------------------------------- forward
    def forward(self, *args, **kwargs):
        if self._needs_finalize and self.comm_stream is not None:
            # gradients are about to be accumulated again before the optimizer ran: the next
            # backward's in-place adds into p.grad must follow the packs still reading it
            torch.cuda.current_stream().wait_stream(self.comm_stream)
        if self.sync == "params" and torch.is_grad_enabled():
            self._fwd_samples += _leading_dim(args, kwargs)
        if self.cast_dtype is not None or self.channels_last:
            args = _cast_inputs(args, self.cast_dtype, self.channels_last)
            kwargs = _cast_inputs(kwargs, self.cast_dtype, self.channels_last)
        return self.module(*args, **kwargs)

    def train_step(self, inputs, targets=None, loss_fn=None, microbatches: int = 1):
        """Forward + backward of one (optionally micro-batched) step; same protocol as
        ``PipelineEngine.train_step`` so scripts can switch strategy without changes."""
        from ..ops import scaled_loss

        fn = loss_fn or getattr(self, "loss_fn", None)
        if fn is None:
            raise ValueError("train_step needs loss_fn= (or model.loss_fn)")
        xs = inputs.chunk(microbatches)
        ts = targets.chunk(microbatches) if targets is not None else [None] * len(xs)
        total = None
        for i, (x, t) in enumerate(zip(xs, ts)):
            ctx = self.no_sync() if i < len(xs) - 1 else contextlib.nullcontext()
            with ctx:
                loss = scaled_loss(fn, self(x), t, 1.0 / len(xs))
                loss.backward()
            total = loss.detach() if total is None else total + loss.detach()
        return total

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (microbatching) without reducing."""
        prev = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = prev

    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, sd, strict: bool = True):
        res = self.module.load_state_dict(sd, strict=strict)
        self.space.sync_master_from_model()
        return res

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks.clear()

    def extra_repr(self) -> str:
        period = f"{self.sync_samples} samples" if self.sync_samples else self.sync_every
        return (f"world={self.world}, sync={self.sync}, period={period}, "
                f"buckets={len(self.space.buckets)}, overlap={self.comm_stream is not None}")


def log_plan(engine: DataParallel):
    log = get_logger()
    for bk in engine.space.buckets:
        log.info("bucket %d: %s x %d params, %.1f MB (reduce %s)", bk.index, bk.dtype, len(bk.params),
                 bk.numel * torch.tensor([], dtype=bk.grad_dtype).element_size() / 2**20, bk.grad_dtype)
