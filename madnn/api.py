"""Public API: ``distribute``, the reference-compatible ``parallelize`` /
``synchronize_model``, and the ``Trainer``.

Reference crosswalk:

=====================================================  =====================================
reference (Lua)                                        madnn
=====================================================  =====================================
``mpi.start(true)`` (README.md:33-34)                  ``madnn.init()`` (implicit)
``parallelize(data, labels, model, size, mpi, mpinn,   ``madnn.parallelize(data, targets, model,
batchSize)`` (datamodule.lua:15-53)                    size=None, sync_every=None)``
``parallelize(..., -1)`` + ``synchronizeModel``        ``sync_every=-1`` + ``madnn.synchronize_model``
(README.md:66-75; datamodule.lua:211-224)
patched ``nn.StochasticGradient:train``               ``madnn.Trainer``
(datamodule.lua:117-184)
—                                                      ``madnn.distribute(model, opt, strategy=...)``
=====================================================  =====================================
"""
from __future__ import annotations

import math
import time
from typing import Callable, Optional, Sequence

import torch
from torch import nn

from . import comm, ops
from . import runtime as rt
from .config import Config, torch_dtype
from .parallel.dp import DataParallel, default_sync_period, robustness_tick
from .parallel.flat import FlatParamSpace
from .utils.logging import get_logger

NORM_TYPES = (nn.BatchNorm1d, nn.BatchNorm2d, nn.BatchNorm3d, nn.SyncBatchNorm, nn.LayerNorm, nn.GroupNorm,
              nn.InstanceNorm2d)


def _is_norm_module(m: nn.Module) -> bool:
    if isinstance(m, NORM_TYPES):
        return True
    name = type(m).__name__.lower()
    return "norm" in name


def _norm_param_ids(model: nn.Module) -> set:
    ids = set()
    for m in model.modules():
        if _is_norm_module(m):
            for p in m.parameters(recurse=False):
                ids.add(id(p))
    return ids


def _has_conv(model: nn.Module) -> bool:
    return any(isinstance(m, (nn.Conv2d,)) for m in model.modules())


def _is_fused(opt) -> bool:
    from .optim import _FlatOptimizer

    return isinstance(opt, _FlatOptimizer)


def prepare_model(model: nn.Module, cfg: Config, device: torch.device):
    """Move the model to its device and decide dtype / layout per parameter."""
    model.to(device)
    dtype = torch_dtype(cfg.dtype) if device.type == "cuda" else torch.float32
    if "cpu_dtype" in cfg.extra and device.type == "cpu":
        dtype = torch_dtype(cfg.extra["cpu_dtype"])
    norm_ids = _norm_param_ids(model) if cfg.keep_fp32_norms else set()
    cl = cfg.channels_last if cfg.channels_last is not None else (device.type == "cuda" and _has_conv(model))
    if cl:
        model.to(memory_format=torch.channels_last)

    def dtype_of(p):
        return torch.float32 if id(p) in norm_ids else dtype

    return dtype, dtype_of, cl


def build_space(model: nn.Module, optimizer, cfg: Config, device, dtype_of, channels_last: bool):
    if optimizer is not None:
        groups = [g["params"] for g in optimizer.param_groups]
    else:
        groups = [[p for p in model.parameters() if p.requires_grad]]
    mb = cfg.bucket_mb
    if not mb:
        from .config import auto_bucket_mb

        rb = 4 if cfg.reduce_dtype in ("float32", "fp32") else 2
        mb = auto_bucket_mb(sum(p.numel() for g in groups for p in g if p.requires_grad) * rb)
    return FlatParamSpace(groups, dtype_of=dtype_of, bucket_cap_mb=mb,
                          reduce_dtype=None if cfg.reduce_dtype == "auto" else torch_dtype(cfg.reduce_dtype),
                          device=device,
                          channels_last_of=(lambda p: channels_last and p.dim() == 4))


def plan(model: nn.Module, optimizer=None, *, strategy: str = "auto", config: Optional[Config] = None,
         example_input=None, **kwargs):
    """The planner's placement for ``model`` on this job (``madnn.planner.Plan``) without applying
    it: trace, cost (measured on the job's GPUs) and, at W > 1, the measured links.  Pass it back
    with ``distribute(model, opt, plan=p)`` to use it, or inspect ``p.describe()`` /
    ``p.table()`` first."""
    from .planner import plan_model

    cfg = config or Config.from_env(**kwargs)
    cfg.strategy = strategy
    rt.init(timeout_s=cfg.timeout_s)
    _swap_kernels(model, cfg)
    return plan_model(model, cfg, world=rt.get_world_size(), example_input=example_input, optimizer=optimizer)


def _swap_kernels(model: nn.Module, cfg: Config) -> None:
    device = rt.device()
    if cfg.fused_kernels == "on" or (cfg.fused_kernels == "auto" and device.type == "cuda"):
        from .nn.swap import use_madnn_kernels

        swapped = use_madnn_kernels(model)
        if swapped:
            get_logger().info("madnn: hand-written kernels swapped in: %s", swapped)


def distribute(model: nn.Module, optimizer=None, *, strategy: Optional[str] = None, config: Optional[Config] = None,
               example_input=None, loss_fn: Optional[Callable] = None, plan=None, **kwargs):
    """Place ``model`` across the GPUs of this node and return ``(engine, optimizer)``.

    ``strategy``: ``"auto"`` (the planner traces and costs the model and picks
    DP, PP or DP x PP for the available ranks and 288 GB per GPU), or force
    ``"dp"``, ``"pp"``, ``"dp_pp"``, ``"tp"``.  ``plan``: a placement from
    :func:`plan` to apply as is (no re-planning).  ``kwargs`` override
    :class:`~madnn.config.Config` fields (e.g. ``bucket_mb=32``,
    ``pp_stages=4``, ``microbatches=8``, ``dtype="bfloat16"``).
    """
    cfg = config or Config.from_env(**kwargs)
    if strategy is not None:
        cfg.strategy = strategy
    rt.init(timeout_s=cfg.timeout_s)
    apply_debug_flags(cfg)
    device = rt.device()
    _swap_kernels(model, cfg)
    strat = cfg.strategy
    if plan is not None:
        strat = plan.strategy
        if strat == "tp":
            cfg.tp_size = plan.tp
    elif strat in ("auto", "pp", "dp_pp"):
        from .planner import plan_model

        try:
            plan = plan_model(model, cfg, world=rt.get_world_size(), example_input=example_input,
                              optimizer=optimizer)
        except Exception as e:  # noqa: BLE001 - an uncostable model still trains data-parallel
            if strat != "auto":
                raise
            get_logger().warning("madnn planner could not cost the model (%s); using data parallelism", e)
            plan = None
        if plan is not None:
            strat = plan.strategy
            if strat == "tp":
                cfg.tp_size = plan.tp
        else:
            strat = "dp"
    if strat in ("pp", "dp_pp"):
        from .parallel.pp import build_pipeline

        return build_pipeline(model, optimizer, cfg, plan, loss_fn=loss_fn)
    if strat == "tp":
        from .parallel.tp import apply_tensor_parallel

        engine, optimizer = apply_tensor_parallel(model, optimizer, cfg)
        engine.plan = plan
        return engine, optimizer
    if strat == "none":
        return model, optimizer
    engine, optimizer = _distribute_dp(model, optimizer, cfg, device, loss_fn=loss_fn, plan=plan)
    return engine, optimizer


def apply_debug_flags(cfg: Config) -> None:
    """Wire the debug/robustness switches of ``cfg`` into the subsystems that implement them:
    ``debug_shapes`` (reference ``printDims``, nodemodule.lua:3) turns on the per-layer shape
    trace of the tensor-parallel layers; ``check_collectives`` turns on the collective-order
    fingerprint that the engines compare across ranks every ``MADNN_CHECK_EVERY`` steps."""
    from .parallel.tp import set_debug_shapes

    if cfg.debug_shapes:
        set_debug_shapes(True)
    if cfg.check_collectives and not comm.order_check_enabled():
        comm.enable_order_check(True)


def enable_checkpointing(module: nn.Module) -> None:
    """Activation checkpointing for one module, instance-level (state-dict keys and hooks unchanged)."""
    if getattr(module, "_madnn_ckpt_forward", None) is not None:
        return
    orig = module.forward

    def fwd(*args, **kwargs):
        if module.training and torch.is_grad_enabled():
            return torch.utils.checkpoint.checkpoint(orig, *args, use_reentrant=False, **kwargs)
        return orig(*args, **kwargs)

    module._madnn_ckpt_forward = orig
    module.forward = fwd


def _apply_checkpointing(model: nn.Module, cfg: Config, plan) -> int:
    flags = None
    layers = None
    if plan is not None and plan.spine is not None and plan.spine.source in ("declared", "sequential", "hf"):
        layers, flags = plan.spine.layers, plan.checkpoint
    elif cfg.checkpointing == "all":
        from .planner.trace import trace

        sp = trace(model)
        if sp.source in ("declared", "sequential", "hf"):
            layers = sp.layers
            flags = [0 < i < len(layers) - 1 or len(layers) == 1 for i in range(len(layers))]
    if not layers or not flags:
        return 0
    n = 0
    for layer, f in zip(layers, flags):
        if f:
            enable_checkpointing(layer)
            n += 1
    return n


def _distribute_dp(model, optimizer, cfg: Config, device, group=None, src_rank: int = 0, loss_fn=None, plan=None):
    from .parallel.pp import materialize_

    # a model built on the meta device (e.g. 8B weights never held on the host) is allocated
    # straight on this rank's GPU; the optimizer is re-pointed at the real parameters
    if materialize_(model, device, getattr(model, "init_weights", None), optimizer):
        get_logger().info("madnn: materialised meta-device model on %s", device)
    nck = _apply_checkpointing(model, cfg, plan) if cfg.checkpointing != "none" else 0
    if nck:
        get_logger().info("madnn: activation checkpointing on %d layers", nck)
    dtype, dtype_of, cl = prepare_model(model, cfg, device)
    fused = optimizer is None or _is_fused(optimizer)
    space = build_space(model, optimizer, cfg, device, dtype_of, cl)
    world = rt.get_world_size(group)
    sync, sync_every, sync_samples = cfg.sync, cfg.sync_every, None
    if sync == "params" and sync_every == -1:
        sync = "manual"  # the reference's batchSize = -1 (datamodule.lua:45)
    if sync == "params" and sync_every is None:
        sync_samples = _heuristic_period(cfg, group, device)
    engine = DataParallel(model, space, group=group, src_rank=src_rank, sync=sync,
                          sync_every=sync_every if sync_every not in (None, -1) else 1,
                          sync_samples=sync_samples, sync_budget=cfg.sync_budget,
                          overlap=cfg.overlap, cast_dtype=dtype, channels_last=cl, unpack_grads=not fused,
                          broadcast_buffers=cfg.broadcast_buffers, find_unused=cfg.find_unused,
                          sync_comm=cfg.sync_comm, rebuild_buckets=cfg.rebuild_buckets and fused)
    engine.loss_fn = loss_fn or getattr(model, "loss_fn", None)
    engine.plan = plan
    if optimizer is not None:
        if fused:
            optimizer.bind(space)
            optimizer.grad_source = engine
            optimizer.nonfinite = cfg.nonfinite
            engine.optimizer = optimizer
        else:
            if cfg.sync == "grads":
                optimizer.register_step_pre_hook(lambda *a, **k: engine.finalize_grads())
            optimizer.register_step_post_hook(lambda *a, **k: _after_plain_step(engine))
    get_logger().info("madnn dp: world=%d buckets=%d params=%.1fM dtype=%s channels_last=%s", world,
                      len(space.buckets), space.numel() / 1e6, dtype, cl)
    return engine, optimizer


def _heuristic_period(cfg: Config, group=None, device=None) -> int:
    """The reference's default period (R6, datamodule.lua:68-78) for ``sync="params"`` without
    ``sync_every``: 1/10/50/100 SAMPLES by the size of the shard -- ``cfg.local_size``, else the
    shard ``madnn.data`` last cut on this rank.  With neither, the shard is taken to be large (the
    heuristic's top tier, 100 samples).  The period is AGREED over the group (the smallest shard
    decides): with ``remainder="last"`` shards differ in size and may fall into different tiers,
    and ranks that averaged at different steps would pair up unrelated collectives."""
    from .data import last_local_size

    local = cfg.local_size if cfg.local_size is not None else last_local_size()
    if local is None:
        get_logger().warning("madnn dp: sync='params' without sync_every and no known shard size "
                             "(pass local_size=): using the heuristic's top tier, 100 samples")
    v = int(local) if local is not None else 10 ** 9
    if not comm._local(group) and rt.get_world_size(group) > 1:
        t = torch.tensor([-float(v)], dtype=torch.float64, device=device)
        comm.all_reduce(t, "max", group=group)
        v = int(-t.item())
    return default_sync_period(v)


def _after_plain_step(engine: DataParallel):
    engine.space.sync_master_from_model()
    engine.after_step()


# --------------------------------------------------------------------------
# Reference-compatible surface
# --------------------------------------------------------------------------
def _flat_collective(tensors, op: str, group=None, src: int = 0, scale: float = 1.0) -> int:
    """One collective per (device, dtype) class of ``tensors``: K4 pack into a flat buffer, the
    collective chosen by the selector (R9), K4 unpack with ``scale`` fused.  A broadcast moves
    the class's own dtype (a bf16 model moves bf16 bytes: the values are copied, not combined);
    a SUM all-reduce packs into fp32 (the K4 cast is free), so a bf16 model's W-rank sum is not
    rounded to bf16 before the 1/W scale.  Returns the number of collectives issued."""
    classes = {}
    for t in tensors:
        if t is not None:
            classes.setdefault((t.device, t.dtype), []).append(t)
    n_calls = 0
    for (dev, dt), ts in sorted(classes.items(), key=lambda kv: (str(kv[0][0]), str(kv[0][1]))):
        offs, n = [], 0
        for t in ts:
            offs.append(n)
            n += (t.numel() + 15) // 16 * 16
        fdt = dt if (dt.is_floating_point and op == "broadcast") else torch.float32
        flat = torch.zeros(n, dtype=fdt, device=dev)
        ops.bucket_pack(ts, flat, offs, 1.0)
        coll = comm.select(flat, op, group)
        if op == "broadcast":
            coll(flat, src=src, group=group)
        else:
            coll(flat, "sum", group=group)
        ops.bucket_unpack(ts, flat, offs, scale)
        n_calls += 1
    return n_calls


def synchronize_model(model: nn.Module, group=None, params: bool = True, grads: bool = True) -> None:
    """Average every parameter and gradient across ranks (R10, datamodule.lua:211-224).

    Bucketed: one K4 pack, one all-reduce (through the collective selector, R9) and one
    K4 unpack (1/W fused) per (device, dtype) class instead of one blocking collective per
    tensor."""
    if comm._local(group):
        return
    world = rt.get_world_size(group)
    if isinstance(model, DataParallel):
        model = model.module
    with torch.no_grad():
        if params:
            # parameters homed in a flat space (a fused optimizer's) are averaged through their
            # fp32 masters -- one all-reduce per bucket, no pack -- and the compute copies are
            # re-derived; the rest go through the dtype-class flat collective
            plain, spaces = [], {}
            for p in model.parameters():
                home = getattr(p, "_madnn_home", None)
                if home is not None and id(p) in home.param_info:
                    spaces[id(home)] = home
                else:
                    plain.append(p)
            for sp in spaces.values():
                for bk in sp.buckets:
                    coll = comm.select(bk.master, "all_reduce", group)
                    coll(bk.master, "sum", group=group)
                    bk.master.mul_(1.0 / world)
                sp.sync_model_from_master()
            _flat_collective(plain, "all_reduce", group, scale=1.0 / world)
        if grads:
            _flat_collective([p.grad for p in model.parameters()], "all_reduce", group, scale=1.0 / world)


class _PeriodicSync:
    """Auto-sync (R7): average parameters and gradients every ``period`` SAMPLES of the root
    model's training, counted as the reference counts them (datamodule.lua:102,151: one per
    backward / trainer step of a single example).  A backward over a minibatch advances the
    counter by its batch size when the caller says how many samples it held
    (:meth:`count_next`; ``Trainer`` does), otherwise by one.  The sync fires whenever the counter
    crosses a multiple of the period.  Hooks go on the root's own parameters only -- no
    class-wide monkey patch (SURVEY A-8), so nested containers cannot double-sync."""

    def __init__(self, model: nn.Module, period: int, local_size: int, group=None):
        self.model, self.period, self.local_size, self.group = model, period, local_size, group
        self.counter = 0          # samples seen
        self.backwards = 0
        self.syncs = 0
        self._next = None
        self._armed = False
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in model.parameters()
                       if p.requires_grad]

    def count_next(self, samples: int) -> None:
        """The next backward pass covers ``samples`` samples (minibatch training)."""
        self._next = int(samples)

    def _hook(self, _p):
        if not self._armed:
            self._armed = True
            torch.autograd.Variable._execution_engine.queue_callback(self._on_end)

    def _on_end(self):
        self._armed = False
        n = self._next if self._next is not None else 1
        self._next = None
        before = self.counter
        self.counter += n
        self.backwards += 1
        if self.counter // self.period > before // self.period:
            self.sync()

    def sync(self):
        synchronize_model(self.model, self.group)
        self.syncs += 1

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


_USAGE = ("usage: madnn.parallelize(data, targets, model, size=None, sync_every=None)\n"
          "  data/targets: sliceable datasets; model: nn.Module; size: dataset size (default len(data));\n"
          "  sync_every: sync period in SAMPLES, as the reference counts (None = heuristic, -1 = manual)")


def parallelize(data, targets, model: nn.Module, size: Optional[int] = None, sync_every: Optional[int] = None, *,
                remainder: str = "drop", shuffle_shards: bool = False, group=None, verbose: bool = True):
    """One-call data parallelism (R2, datamodule.lua:15-53).

    Starts the communicator, broadcasts the initial parameters from rank 0
    (always — SURVEY A-6), shards ``data``/``targets`` into contiguous stripes
    (R5), and unless ``sync_every == -1`` (manual mode, R12) installs periodic
    synchronisation of parameters and gradients every ``sync_every`` SAMPLES -- the
    reference's unit (its ``batchSize`` argument counts per-example backward calls,
    datamodule.lua:102,151; SURVEY A-1): a minibatch of B samples trained through
    :class:`Trainer` advances the count by B, a bare ``loss.backward()`` by one.  Default:
    the reference heuristic on the local shard size (R6).

    Returns ``(data_shard, target_shard, shard_size)``; on missing arguments
    prints the usage and returns ``-1`` like the reference.  The chosen period
    is available as ``model._madnn_sync.period``.
    """
    if data is None or targets is None or model is None:
        print(_USAGE)
        return -1
    rt.init()
    if size is None:
        size = len(data)
    with torch.no_grad():
        # bucketed broadcast of the initial parameters and buffers (reference
        # synchronizeParameters, datamodule.lua:33, sent one tensor at a time)
        _flat_collective([p.data for p in model.parameters()] + [b for b in model.buffers()
                                                                 if b.is_floating_point()],
                         "broadcast", group, src=0)
        for b in model.buffers():
            if not b.is_floating_point():
                comm.broadcast(b, src=0, group=group)
    from .data import shard

    d = shard(data[:size], remainder=remainder, strided=shuffle_shards, verbose=verbose)
    t = shard(targets[:size], remainder=remainder, strided=shuffle_shards, verbose=False)
    local = len(d)
    if sync_every != -1:
        period = sync_every if sync_every is not None else default_sync_period(local)
        old = getattr(model, "_madnn_sync", None)
        if old is not None:
            old.remove()
        model._madnn_sync = _PeriodicSync(model, period, local, group)
    else:
        model._madnn_sync = None
    rt.barrier(group)
    return d, t, local


class Trainer:
    """Minibatch SGD trainer with the reference trainer's knobs and hooks (R8,
    datamodule.lua:117-184): ``learning_rate``, ``learning_rate_decay``, ``max_iteration``
    (epochs; ``<= 0`` = no limit, stop by raising ``StopIteration`` from ``on_iteration``),
    ``shuffle``, ``on_example`` (after every minibatch; reference ``hookExample``) and
    ``on_iteration(trainer, iteration, error)`` (after every epoch, 1-based ``iteration``;
    ``hookIteration``).  Synchronisation is whatever the
    model carries: a ``parallelize`` periodic hook, a ``distribute`` engine, or nothing.

    Reference fidelity:

    * the default optimizer is :class:`madnn.optim.FusedSGD` over a flat parameter space -- the
      K1 kernel, one launch per bucket, standing in for the reference's fused
      gradient-into-weight ``accUpdateGradParameters`` (datamodule.lua:142);
    * learning-rate schedule exactly as the reference's (datamodule.lua:176-177): the first
      epoch runs at ``learning_rate``; the counter is incremented BEFORE the decay is applied,
      so epoch k >= 2 (1-based) runs at ``learning_rate / (1 + k * decay)``;
    * ``shuffle=True`` draws ONE permutation before the first epoch and keeps it, as the
      reference does (datamodule.lua:123); ``shuffle="epoch"`` redraws it every epoch.
    """

    def __init__(self, model: nn.Module, criterion: Callable, optimizer=None, *, learning_rate: float = 0.01,
                 learning_rate_decay: float = 0.0, max_iteration: int = 25, shuffle=True,
                 batch_size: int = 32, on_example: Optional[Callable] = None,
                 on_iteration: Optional[Callable] = None, verbose: bool = True, device=None,
                 metrics_path: Optional[str] = None):
        self.model, self.criterion = model, criterion
        self.learning_rate, self.learning_rate_decay = learning_rate, learning_rate_decay
        self.max_iteration, self.shuffle, self.batch_size = max_iteration, shuffle, batch_size
        self.on_example, self.on_iteration, self.verbose = on_example, on_iteration, verbose
        self.device = device
        if optimizer is None:
            from .optim import FusedSGD

            optimizer = FusedSGD([p for p in model.parameters() if p.requires_grad], lr=learning_rate)
        self.optimizer = optimizer
        self.epoch = 0          # completed epochs (checkpointed with the trainer state)
        self.cursor = 0         # samples of the current epoch already trained on
        self._partial = (0.0, 0)
        self._order = None
        self.history = []
        self.global_step = 0
        self.meter = None
        if metrics_path:  # per-step JSONL metrics
            from .utils.metrics import StepMeter

            self.meter = StepMeter(model if hasattr(model, "comm_metrics") else None,
                                   samples_per_step=batch_size, path=metrics_path)

    def _lr(self, epoch: int) -> float:
        """Learning rate of 0-based ``epoch`` (reference: 1-based iteration i uses lr for i = 1,
        lr / (1 + i * decay) for i >= 2)."""
        if epoch == 0:
            return self.learning_rate
        return self.learning_rate / (1.0 + (epoch + 1) * self.learning_rate_decay)

    def _perm(self, n: int):
        if not self.shuffle:
            return torch.arange(n)
        if self.shuffle == "epoch" or self._order is None or len(self._order) != n:
            self._order = torch.randperm(n)
        return self._order

    def state_dict(self) -> dict:
        """Resume state (no optimizer: ``madnn.ckpt`` stores that by parameter name): epoch,
        position inside it, step counter, the permutation, the partial epoch error."""
        return {"epoch": self.epoch, "cursor": self.cursor, "global_step": self.global_step,
                "history": list(self.history), "order": None if self._order is None else self._order.tolist(),
                "partial": list(self._partial)}

    def load_state_dict(self, sd: dict) -> None:
        self.epoch, self.global_step = int(sd["epoch"]), int(sd["global_step"])
        self.cursor = int(sd.get("cursor", 0))
        self.history = list(sd.get("history", []))
        self._order = torch.tensor(sd["order"]) if sd.get("order") is not None else None
        self._partial = tuple(sd.get("partial", (0.0, 0)))

    def train(self, data, targets) -> list:
        """Epochs over (``data``, ``targets``) in minibatches of ``batch_size``.  ``max_iteration``
        epochs, or -- ``max_iteration <= 0``, as the reference (datamodule.lua:178) -- until
        ``on_iteration`` raises ``StopIteration``.  ``on_iteration(trainer, iteration, error)`` gets
        the 1-based epoch number (reference ``hookIteration(self, iteration, currentError)``,
        datamodule.lua:169-170)."""
        n = len(data)
        log = get_logger()
        epoch = self.epoch
        while self.max_iteration <= 0 or epoch < self.max_iteration:
            lr = self._lr(epoch)
            for g in self.optimizer.param_groups:
                g["lr"] = lr
            order = self._perm(n) if self.cursor == 0 or self._order is None else self._order
            tot, cnt = self._partial if self.cursor else (0.0, 0)
            for s in range(self.cursor, n, self.batch_size):
                idx = order[s:s + self.batch_size]
                x, y = data[idx], targets[idx]
                if self.device is not None:
                    x, y = x.to(self.device), y.to(self.device)
                if self.meter is not None:
                    self.meter.start()
                ps = getattr(self.model, "_madnn_sync", None)
                if ps is not None:
                    ps.count_next(len(idx))  # the period counts samples (reference semantics)
                self.optimizer.zero_grad(set_to_none=True)
                out = self.model(x)
                loss = self.criterion(out, y)
                loss.backward()
                self.optimizer.step()
                self.global_step += 1
                if not hasattr(self.model, "after_step"):
                    # engines tick in their own after_step; a parallelize()-synchronised model
                    # gets the fault-injection / order-check hooks here
                    robustness_tick(self.global_step)
                if self.meter is not None:
                    self.meter.stop(loss, epoch=epoch + 1, lr=lr)
                tot += float(loss.detach()) * len(idx)
                cnt += len(idx)
                self.cursor = s + len(idx)
                self._partial = (tot, cnt)
                if self.on_example is not None:
                    self.on_example(self, (x, y))
            err = tot / max(cnt, 1)
            self.history.append(err)
            ps = getattr(self.model, "_madnn_sync", None)
            if ps is not None and ps.counter % ps.period != 0:
                ps.sync()  # end-of-epoch sync (reference counter == size branch, fixed to every epoch: A-4)
            if self.verbose:
                log.info("# current error = %.6f (epoch %d, lr %.5g)", err, epoch + 1, lr)
            self.epoch = epoch + 1
            self.cursor, self._partial = 0, (0.0, 0)
            epoch += 1
            if self.on_iteration is not None:
                try:
                    self.on_iteration(self, epoch, err)     # 1-based, like the reference
                except StopIteration:
                    return self.history
        if self.verbose:
            log.info("# StochasticGradient: you have reached the maximum number of iterations")
            log.info("# training error = %.6f", self.history[-1] if self.history else float("nan"))
        return self.history
