"""Graph tracer: turn an arbitrary ``nn.Module`` into a linear spine of layers.

The reference has no tracer — model parallelism needs manual layer
substitution (README.md:89-101).  The planner needs a sequence of callables
``L_0 .. L_{n-1}`` whose composition equals ``model.forward`` and where each
boundary carries ONE tensor, because that is what a pipeline stage boundary
can send over xGMI.  Three sources, tried in order:

1. ``model.pipeline_layers()`` — the model declares its spine (madnn's zoo);
2. ``nn.Sequential`` — its children;
3. ``torch.fx`` — symbolic trace, then cut the graph at every node where
   exactly one tensor value is live across the cut; the segments between cuts
   become ``fx.GraphModule`` layers that share the original parameters (tied
   weights stay tied).
4. Hugging Face models (``madnn.models.hf``): embedding -> ``transformer.h`` /
   ``model.layers`` / ``bert.encoder.layer`` -> head, wrapped as single-tensor layers.
5. Fallback for untraceable models: the module tree's largest ``ModuleList``
   of identical blocks (``transformer.h``, ``model.layers``, ``encoder.layer``)
   is reported for costing, and the model is treated as one layer.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import torch
from torch import fx, nn


@dataclass
class Spine:
    layers: List[nn.Module]
    names: List[str]
    source: str
    block_list: Optional[str] = None  # dotted name of the repeated-block ModuleList, if found
    notes: List[str] = field(default_factory=list)

    def __len__(self):
        return len(self.layers)


class FxSegment(nn.Module):
    """A contiguous slice of an fx graph with one tensor in and one out."""

    def __init__(self, root: nn.Module, graph: fx.Graph, name: str):
        super().__init__()
        self.gm = fx.GraphModule(root, graph, class_name=name)

    def forward(self, x):
        return self.gm(x)


def find_block_list(model: nn.Module) -> Optional[str]:
    best, best_n = None, 1
    for name, m in model.named_modules():
        if isinstance(m, nn.ModuleList) and len(m) > best_n:
            types = {type(c) for c in m}
            if len(types) == 1:
                best, best_n = name, len(m)
    return best


class _Tracer(fx.Tracer):
    """fx tracer that keeps madnn's fused-kernel modules (and torch.nn) as leaves."""

    def is_leaf_module(self, m: nn.Module, qualname: str) -> bool:
        if type(m).__module__.startswith("madnn.nn"):
            return True
        return super().is_leaf_module(m, qualname)


def symbolic_trace(model: nn.Module) -> fx.GraphModule:
    graph = _Tracer().trace(model)
    return fx.GraphModule(model, graph, model.__class__.__name__)


def _fx_split(model: nn.Module) -> Optional[Spine]:
    try:
        gm = symbolic_trace(model)
    except Exception as e:  # noqa: BLE001
        return Spine([model], ["model"], "whole", find_block_list(model), [f"fx trace failed: {type(e).__name__}"])
    nodes = list(gm.graph.nodes)
    placeholders = [n for n in nodes if n.op == "placeholder"]
    if len(placeholders) != 1:
        return Spine([model], ["model"], "whole", find_block_list(model), ["fx: model takes != 1 input"])
    body = [n for n in nodes if n.op not in ("placeholder", "output")]
    out_node = [n for n in nodes if n.op == "output"][0]
    index = {n: i for i, n in enumerate(body)}
    last_use = {}
    for n in body + [out_node]:
        for a in n.all_input_nodes:
            last_use[a] = max(last_use.get(a, -1), index.get(n, len(body)))
    # a cut after body[i] is valid if exactly one value defined at <= i is used at > i
    # (get_attr values are parameters: re-materialised in each segment)
    cuts = []
    live = set(placeholders)
    for i, n in enumerate(body):
        live.add(n)
        live = {v for v in live if last_use.get(v, -1) > i}
        tensor_live = [v for v in live if v.op != "get_attr"]
        if len(tensor_live) == 1 and tensor_live[0] is n and i < len(body) - 1:
            if n.op in ("call_module", "call_function", "call_method"):
                cuts.append(i)
    if not cuts:
        return Spine([model], ["model"], "whole", find_block_list(model), ["fx: no single-tensor cut"])
    # merge cuts so each segment holds at least one call_module or heavy op
    segs, start = [], 0
    for c in cuts + [len(body) - 1]:
        seg = body[start:c + 1]
        if any(x.op == "call_module" for x in seg) or c == len(body) - 1:
            segs.append(seg)
            start = c + 1
    layers, names = [], []
    for k, seg in enumerate(segs):
        g = fx.Graph()
        env = {}
        inputs = set()
        for n in seg:
            for a in n.all_input_nodes:
                if a not in seg and a.op != "get_attr":
                    inputs.add(a)
        if len(inputs) != 1:
            return Spine([model], ["model"], "whole", find_block_list(model), ["fx: segment arity != 1"])
        (inp,) = inputs
        env[inp] = g.placeholder("x")
        for n in seg:
            for a in n.all_input_nodes:
                if a.op == "get_attr" and a not in env:
                    env[a] = g.get_attr(a.target)
            env[n] = g.node_copy(n, lambda a: env[a])
        g.output(env[seg[-1]])
        layers.append(FxSegment(gm, g, f"Segment{k}"))
        names.append(f"seg{k}:{seg[0].name}..{seg[-1].name}")
    return Spine(layers, names, "fx", find_block_list(model))


def trace(model: nn.Module) -> Spine:
    if hasattr(model, "pipeline_layers"):
        layers = list(model.pipeline_layers())
        names = []
        lookup = {id(m): n for n, m in model.named_modules()}
        for i, l in enumerate(layers):
            names.append(lookup.get(id(l), f"layer{i}"))
        return Spine(layers, names, "declared", find_block_list(model))
    if isinstance(model, nn.Sequential):
        return Spine(list(model), [n for n, _ in model.named_children()], "sequential")
    from ..models.hf import hf_pipeline_layers

    hf = hf_pipeline_layers(model)
    if hf is not None:
        bl = find_block_list(model)
        return Spine(hf, [f"{type(l).__name__}{i}" for i, l in enumerate(hf)], "hf", bl)
    return _fx_split(model)


def run_spine(spine: Spine, x):
    for l in spine.layers:
        x = l(x)
    return x
