"""madnn — MI355X-native automatic distributed training.

One call places a model on the GPUs of a node: ``madnn.distribute(model, opt)``
(data-, pipeline- or hybrid-parallel, chosen by a cost model for 288 GB of
HBM3E per GPU), with bucketed RCCL gradient averaging overlapped on HIP
streams and hand-written gfx950 kernels for the optimizer step, LayerNorm and
bucket flatten/unflatten.  The reference library's API (``parallelize``,
``synchronize_model``, the trainer and the ``MP*`` model-parallel layers) is
kept under the same names.
"""
from .config import Config
from .runtime import init, shutdown, get_rank, get_world_size, device, barrier, seed_all
from .api import distribute, plan, parallelize, synchronize_model, Trainer
from . import ops, optim, data, comm, models
from .ckpt import save, load, consolidate

__version__ = "0.1.0"

__all__ = [
    "plan",
    "Config", "init", "shutdown", "get_rank", "get_world_size", "device", "barrier", "seed_all",
    "distribute", "parallelize", "synchronize_model", "Trainer", "ops", "optim", "data", "comm", "models",
    "save", "load", "consolidate",
]
