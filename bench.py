#!/usr/bin/env python3
"""madnn headline benchmark (BASELINE.json metric):

  "samples/sec whole-node ResNet-50 DP + GPT-2 PP at 1/2/4/8 MI355X; scaling eff"

Default (the driver's contract) measures BOTH halves of the metric in one run:

* the primary ``value``: ResNet-50, automatic data parallelism
  (``madnn.distribute``), bf16 compute with fp32 master weights and fp32 BatchNorm,
  channels_last, FusedSGD (momentum 0.9, wd 5e-5) on the hand-written gfx950 kernel,
  bucketed RCCL all-reduce overlapped with backward; 2048 images per GPU (weak scaling, 80 GB
  of the 288 GB HBM; same-box A/Bs: 10.80k img/s at 512 vs 11.37k at 1024,
  profiles/r2_resnet_b1024.md; 11.38k at 1024 vs 11.59k at 1536, profiles/r2_resnet_b1536.md;
  12.65k at 1536 vs 12.85k at 2048, profiles/r2_resnet_b2048.md);
* ``gpt2_pp``: GPT-2 medium (seq 1024, bf16, FusedAdam), pipeline parallel over
  RCCL P2P -- ``pp2`` at 2 GPUs, ``pp4`` at 4, ``dp2 x pp4`` at 8; data parallel at 1 GPU
  (a pipeline needs two stages); 128 sequences per GPU (weak scaling).  The schedule (GPipe,
  1F1B, interleaved with 2 or 4 chunks per rank) and the microbatch count are the planner's
  choice (``--schedule auto``): it prices every variant with layer costs measured on the
  GPUs of the job (per-call fixed cost + per-sample slope, so small microbatches pay for
  their lower GEMM efficiency: profiles/r2_gpt2m_dp1_batch_sweep.jsonl, 4 / 8 / 16 / 32 / 64
  sequences: 194k / 235k / 277k / 308k / 326k tok/s) against the simulated bubble.
  ``--schedule`` / ``--microbatches`` / ``--gpt2-mb`` pin them by hand.

Synthetic data and random init (no network on the box).  ``--model resnet50`` /
``--model gpt2-medium`` run one half only.  Without a launcher environment the
process still joins a world-1 RCCL group (``--no-pg`` disables it), so the 1-GPU
number is taken on the same communicator / reducer path as the 8-GPU one.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Times exactly K steps between a barrier + device synchronize on both sides,
takes the MAX over ranks, and rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

# the hosts' drivers support only dmabuf IPC: RCCL's cross-process buffers need the non-legacy mode,
# set before the HSA runtime initialises (a launcher that exports it already wins)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn.functional as F  # noqa: E402

METRIC = "samples/sec whole-node ResNet-50 DP + GPT-2 PP at 1/2/4/8 MI355X; scaling eff"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="all", choices=["all", "resnet50", "gpt2-medium", "bert-large", "llama3-8b"],
                    help="all (the driver's contract: ResNet-50 + GPT-2), one half of it, or one of BASELINE's other "
                         "configs: bert-large (config 5) / llama3-8b (config 4), planned by madnn.distribute "
                         "(strategy and activation checkpointing are the planner's)")
    ap.add_argument("--tf-config", default=None,
                    help="bert / llama size for --model bert-large|llama3-8b (default: that model; bert-tiny / "
                         "llama3-tiny for CPU harness tests)")
    ap.add_argument("--tf-batch-per-gpu", type=int, default=None,
                    help="sequences per GPU for --model bert-large (default 128 at --seq-len 512) / llama3-8b "
                         "(default 4 at --seq-len 4096)")
    ap.add_argument("--checkpointing", default="auto", choices=["auto", "all", "none"],
                    help="--model bert-large|llama3-8b: activation checkpointing (auto: the planner's per-block "
                         "choice; all / none pin it, for A/Bs)")
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (resnet50)")
    ap.add_argument("--gpt2-batch-per-gpu", type=int, default=128,
                    help="GPT-2 sequences per GPU (global = this x N); 128: 369k tok/s vs 360k at 64 on one "
                         "MI355X, 130 of 288 GB (profiles/r4_batch_size_resnet3072_gpt2_128_96.json)")
    ap.add_argument("--gpt2-config", default="gpt2-medium", help="GPT-2 size (gpt2-tiny for CPU harness tests)")
    ap.add_argument("--gpt2-mb", type=int, default=0,
                    help="GPT-2 sequences per pipeline microbatch (0: the planner picks the microbatch count)")
    ap.add_argument("--gpt2-steps", type=int, default=None, help="GPT-2 timed steps (default: --steps)")
    ap.add_argument("--gpt2-warmup", type=int, default=None, help="GPT-2 warmup steps (default: --warmup)")
    ap.add_argument("--schedule", default="auto",
                    help="pipeline schedule (auto: the planner prices gpipe / 1f1b / interleaved V=2,4 at every "
                         "microbatch count and picks the cheapest | gpipe | 1f1b | interleaved)")
    ap.add_argument("--strategy", default="auto",
                    help="ResNet-50 placement: auto (the planner's choice, BASELINE's 'auto data-parallel') or a "
                         "pinned dp | pp | dp_pp | tp")
    ap.add_argument("--gpt2-strategy", default="auto",
                    help="GPT-2 placement: auto (planner; only the stage count is pinned) or pp / dp_pp")
    ap.add_argument("--graph", type=int, default=0,
                    help="ResNet-50: replay the whole training step as one hipGraph (madnn.utils.graphs)")
    ap.add_argument("--no-pg", action="store_true", help="no world-1 process group when run without a launcher")
    ap.add_argument("--bucket-mb", type=float, default=None)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--channels-last", type=int, default=1)
    ap.add_argument("--seq-len", type=int, default=None, help="default 1024 (GPT-2), 512 (BERT), 4096 (Llama)")
    ap.add_argument("--microbatches", type=int, default=None)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--device", default="cuda", help="cuda (MI355X) or cpu (gloo; for testing the harness)")
    ap.add_argument("--backend", default=None,
                    help="process-group backend override (default: nccl=RCCL on cuda, gloo on cpu); gloo on cuda "
                         "lets tests run several ranks on one GPU, which RCCL refuses")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--std-batch", type=int, default=512,
                    help="also time ResNet-50 at this standard per-GPU batch (config.std_batch; 0 = skip)")
    ap.add_argument("--gpt2-timeout", type=float, default=420.0,
                    help="seconds the GPT-2 phase may take before it is reported as an error (below the 600 s "
                         "process-group timeout, whose watchdog would abort the process first)")
    ap.add_argument("--miopen-benchmark", type=int, default=0,
                    help="torch.backends.cudnn.benchmark (MIOpen find).  Both modes read the shipped MI355X "
                         "find-db (madnn/tuning/miopen, seeded by madnn.init), so 0 already runs the tuned solvers")
    return ap.parse_args()


def _sync_all():
    if not torch.cuda.is_available():
        if dist.is_initialized():
            dist.barrier()
        return
    torch.cuda.synchronize()
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()
        torch.cuda.synchronize()


def bench_resnet(args, world, rank):
    import madnn
    from madnn.models import resnet50
    from madnn.optim import FusedSGD

    # 2048 images per GPU: sized for 288 GB HBM3E (80 GB peak), and large enough that the
    # per-step fixed costs (kernel boundaries, MIOpen workspace memsets, the optimizer pass) are
    # amortised (same box: 12650 img/s at 1536 -> 12850 at 2048, profiles/r2_resnet_b2048.md); the
    # shipped find-db holds the tuned solvers for this shape (and for 512 / 1024 / 1536 / 3072);
    # 3072 is slower again: 249 ms/step = 12.3k img/s (profiles/r4_batch_size_resnet3072_gpt2_128_96.json)
    per_gpu = args.batch or 2048
    torch.manual_seed(0)
    model = resnet50()
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    kw = {}
    if args.bucket_mb:
        kw["bucket_mb"] = args.bucket_mb
    # the automatic path (BASELINE "ResNet-50 auto data-parallel"): the planner traces and costs
    # the model on this job's GPUs (and, at N > 1, measures the job's RCCL links) and picks the
    # placement.  The metric is ResNet-50 DATA parallel, whose ranks each draw their own images:
    # a non-DP choice is recorded as rejected and data parallelism runs instead.  --strategy dp
    # pins it without planning.
    kw.update(overlap=not args.no_overlap, channels_last=bool(args.channels_last), global_batch=per_gpu * world)
    example = torch.zeros(1, 3, args.image_size, args.image_size)
    plan, rejected, planned = None, None, None
    if args.strategy == "auto":
        plan = planned = madnn.plan(model, opt, example_input=example, **kw)
        if plan.strategy != "dp":
            rejected, plan = _plan_info(plan), None
            print(f"bench: the planner chose {rejected} for ResNet-50; running data parallel", file=sys.stderr)
    dmodel, opt = madnn.distribute(model, opt, strategy=None if plan is not None else "dp", plan=plan,
                                   example_input=example, **kw)
    dev = madnn.device()
    x, y = madnn.data.synthetic_batch("image", per_gpu, dev, dtype=torch.bfloat16 if dev.type == "cuda" else
                                      torch.float32, channels_last=bool(args.channels_last), seed=1234 + rank,
                                      shape=(3, args.image_size, args.image_size))

    def step():
        out = dmodel(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    tw = time.perf_counter()
    run = step
    if args.graph and dev.type == "cuda":
        # the whole step (forward, backward with the bucketed all-reduce, optimizer) as ONE
        # hipGraph replay: the warm-up steps run eagerly inside capture_step, then one replay
        from madnn.utils.graphs import capture_step

        run = capture_step(step, warmup=max(args.warmup, 3))
        run()
    else:
        for _ in range(args.warmup):
            step()
    _sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = run()
    _sync_all()
    dt = time.perf_counter() - t0
    if run is not step:
        step()   # one eager step after the timed region: its comm events feed comm_metrics
        _sync_all()
    out = (dt, per_gpu * world, {"warmup_s": round(t0 - tw, 1), "model": "resnet50", "global_batch": per_gpu * world,
                                 "graph": run is not step,
                                 "per_gpu_batch": per_gpu, "seq_len": None,
                                 "image": [3, args.image_size, args.image_size],
                                 "parallelism": _parallelism(plan, world),
                                 "optimizer": "FusedSGD(momentum=0.9)", "loss": float(loss.detach()),
                                 "process_group": dist.get_backend() if dist.is_initialized() else None,
                                 "peak_mem_gib": _peak_gib(), "plan": _plan_info(plan), "plan_rejected": rejected,
                                 "tuning_timings": _tuning_timings(), **_comm_fields(dmodel, planned)})
    dmodel.remove_hooks()
    return out


def _parallelism(plan, world: int) -> str:
    if plan is None:
        return f"dp{world}"
    if plan.pp > 1:
        return f"pp{plan.pp}" if plan.dp == 1 else f"dp{plan.dp}xpp{plan.pp}"
    return f"dp{plan.dp}" if plan.tp == 1 else f"dp{plan.dp}xtp{plan.tp}"


def _plan_info(plan):
    """What the planner chose (None when the strategy was pinned without a plan)."""
    if plan is None:
        return None
    return {"strategy": plan.strategy, "dp": plan.dp, "pp": plan.pp, "tp": plan.tp,
            "schedule": plan.schedule if plan.pp > 1 else None, "virtual": plan.virtual if plan.pp > 1 else None,
            "microbatches": plan.microbatches if plan.pp > 1 else None, "est_step_ms": round(plan.est_step_s * 1e3, 2),
            "costs": "measured" if plan.measured else "analytic", "candidates": len(plan.candidates),
            "comm_measured": bool(getattr(plan, "comm_probe", None)),
            "est_mem_gb": round(max(plan.est_mem_gb), 1), "plan_s": round(getattr(plan, "plan_s", 0.0), 1)}


def _tuning_timings():
    import madnn.ops as ops

    return ops.tuning_timings()


def _comm_fields(engine, plan) -> dict:
    """The numbers that explain an N > 1 result: the last step's exposed gradient all-reduce and
    its achieved bus bandwidth (``DataParallel.comm_metrics``), the job-start link probe's
    all-reduce busbw and P2P rate (``comm.probe``, what the planner priced with)."""
    out = {"comm_exposed_ms": None, "busbw_gbps": None, "p2p_gbps": None}
    try:
        m = engine.comm_metrics() if hasattr(engine, "comm_metrics") else {}
    except Exception:  # noqa: BLE001 - metrics never fail the bench
        m = {}
    if m.get("comm_exposed_ms") is not None:
        out["comm_exposed_ms"] = round(m["comm_exposed_ms"], 3)
    if m.get("busbw_gbps") is not None:
        out["busbw_gbps"] = round(m["busbw_gbps"], 2)
    probe = getattr(plan, "comm_probe", None) if plan is not None else None
    if probe:
        out["p2p_gbps"] = round(probe["p2p_gbps"], 2)
        out["probe_allreduce_busbw_gbps"] = round(probe["allreduce_busbw_gbps"], 2)
    if "bubble_fraction" in m:
        out["bubble_fraction"] = round(m["bubble_fraction"], 4)
    if "p2p_bytes" in m:
        out["p2p_bytes"] = m["p2p_bytes"]
    if "plan_lags" in m:
        # the pipeline's issue plans (transfer lag in forward-chunk units), the measured step of
        # each during the warm-up and the one kept (parallel.pp.PipelineEngine._init_plans)
        out["pp_plan"] = {"lags": m["plan_lags"], "kept": m["plan_lag"], "step_ms": m["plan_step_ms"]}
    return out


def gpt2_layout(world: int):
    """(strategy, pp stages, parallelism label) of the GPT-2 half at ``world`` GPUs."""
    if world == 1:
        return "dp", 1, "dp1"
    stages = 4 if world % 4 == 0 else (2 if world % 2 == 0 else world)
    dp = world // stages
    return "pp", stages, (f"pp{stages}" if dp == 1 else f"dp{dp}xpp{stages}")


def bench_gpt2(args, world, rank):
    import madnn
    from madnn.models.gpt2 import GPT2, gpt2_config
    from madnn.optim import FusedAdam

    cfg = gpt2_config(args.gpt2_config)
    gbatch = args.gpt2_batch_per_gpu * world
    strategy, stages, par = gpt2_layout(world)
    dp = world // stages
    per_replica = gbatch // dp
    micro = args.microbatches or (max(per_replica // args.gpt2_mb, 1) if stages > 1 and args.gpt2_mb else None)
    torch.manual_seed(0)
    model = GPT2(cfg)
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
    kw = {}
    if args.schedule and stages > 1:
        sched = args.schedule
        if sched == "interleaved" and micro and micro % stages:
            sched = "1f1b"  # interleaving needs microbatches % stages == 0
        kw["schedule"] = sched
    # the automatic path (BASELINE "GPT-2 medium auto pipeline-parallel, 4 stages"): only the stage
    # count is pinned; the planner picks schedule, microbatches, chunks and checkpointing from
    # layer costs measured on this job's GPUs and (N > 1) the job's measured P2P / all-reduce rates
    engine, opt = madnn.distribute(model, opt, strategy=args.gpt2_strategy if stages > 1 else args.strategy,
                                   pp_stages=stages if stages > 1 else None, microbatches=micro,
                                   checkpointing="none", global_batch=gbatch,
                                   example_input=torch.zeros(1, args.seq_len, dtype=torch.long), **kw)
    plan = getattr(engine, "plan", None)
    if plan is not None and plan.pp != stages:
        raise RuntimeError(f"GPT-2 bench pins {stages} pipeline stages, the planner built {_plan_info(plan)}")
    dev = madnn.device()
    # every dp replica draws its own token batch; pipeline stages of one replica share it
    g = torch.Generator(device="cpu").manual_seed(4321 + (rank // stages))
    ids = torch.randint(0, cfg.vocab_size, (per_replica if stages > 1 else gbatch // world, args.seq_len),
                        generator=g).to(dev)

    accum = {"microbatches": args.microbatches} if stages == 1 and args.microbatches else {}

    def step():
        # 1 GPU: --microbatches M accumulates M microbatches under no_sync, as a pipeline rank
        # computes its share of the step
        loss = engine.train_step(ids, ids, **accum)
        opt.step()
        return loss

    steps = args.gpt2_steps or args.steps
    warm = args.warmup if args.gpt2_warmup is None else args.gpt2_warmup
    # a pipeline engine with two issue plans times them in its steps 1 .. 2L (PipelineEngine.
    # _init_plans); those steps run before the warm-up proper, so the timed steps all use the
    # plan it kept whatever --warmup is
    tuning = 2 * len(getattr(engine, "_lags", [0.0])) if len(getattr(engine, "_lags", [0.0])) > 1 else 0
    extra = max(0, tuning + 1 - warm)
    for _ in range(extra + warm):
        step()
    _sync_all()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step()
    _sync_all()
    dt = time.perf_counter() - t0
    lv = float(loss.detach()) if loss is not None else float("-inf")
    if stages > 1 and dist.is_initialized():   # the last stage holds it: bring it to rank 0
        t = torch.tensor([lv], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lv = float(t.item())
    lv = None if lv == float("-inf") else lv
    held = _heldout_loss(engine, model, cfg.vocab_size, ids.shape, 98765 + rank // stages, stages, rank)
    info = {"model": args.gpt2_config, "global_batch": gbatch, "per_gpu_batch": args.gpt2_batch_per_gpu,
            "seq_len": args.seq_len, "parallelism": par, "microbatches": getattr(engine, "M", 1) if stages > 1 else 1,
            "planned_step_ms": round(engine.plan.est_step_s * 1e3, 2) if getattr(engine, "plan", None) else None,
            "schedule": getattr(engine, "schedule", None) if stages > 1 else None,
            "virtual_stages": getattr(engine, "V", None) if stages > 1 else None,
            "optimizer": "FusedAdam", "steps": steps, "warmup": warm, "plan_tuning_steps": extra,
            "loss_last_stage": lv, "heldout_loss": held, "ln_vocab": round(math.log(cfg.vocab_size), 4),
            "accum_microbatches": args.microbatches if stages == 1 and args.microbatches else None,
            "peak_mem_gib": _peak_gib(), "plan": _plan_info(plan), **_comm_fields(engine, plan)}
    return dt, steps, gbatch, info


def _heldout_loss(engine, model, vocab: int, shape, seed: int, stages: int, rank: int):
    """The loss on a fresh random token batch the model never trained on: forward only, outside
    the timed region (the reference scores its trained net on held-out data,
    cifar_example/sgd-torchad_nn-cifar.lua:266-275).  Next to a low training loss on the one
    repeated batch, a held-out loss near ln(V) says the model memorised it; a low held-out loss
    on a causal model would mean it sees the tokens it predicts.  Pipeline: every rank joins the
    forward, the last stage's value reaches rank 0 (MAX all-reduce)."""
    import madnn

    dev = madnn.device()
    g = torch.Generator(device="cpu").manual_seed(seed)
    ids = torch.randint(0, vocab, tuple(shape), generator=g).to(dev)
    with torch.no_grad():
        out = engine.forward_step(ids) if stages > 1 else engine(ids)
        lv = float(model.loss_fn(out, ids)) if out is not None else float("-inf")
    if stages > 1 and dist.is_initialized():
        t = torch.tensor([lv], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        lv = float(t.item())
    return round(lv, 4) if lv != float("-inf") else None


TF_METRIC = {"bert-large": "tokens/s BERT-large auto-partition + activation checkpointing + fused Adam (BASELINE "
                           "config 5)",
             "llama3-8b": "tokens/s Llama-3 8B auto hybrid DP x PP, 288 GB per-GPU sizing (BASELINE config 4)"}


def bench_transformer(args, world, rank):
    """BASELINE configs 4 and 5 on the same timing contract as the headline: the planner
    (``strategy="auto"``, ``checkpointing="auto"``) places the model on this job's GPUs -- DP, PP
    or DP x PP, and per block whether to recompute activations, priced against 288 GB -- and the
    K steps are bracketed by a barrier + device synchronize, MAX over ranks.  Llama-3 8B is built
    on the meta device and materialised per rank (its stage only under a pipeline plan)."""
    import madnn
    from madnn.optim import FusedAdam

    name = args.model
    seq = args.seq_len
    torch.manual_seed(0)
    if name == "bert-large":
        from madnn.models.bert import BertForPreTraining, bert_config

        cfg = bert_config(args.tf_config or "bert-large")
        model = BertForPreTraining(cfg)
        per_gpu = args.tf_batch_per_gpu or 128
    else:
        from madnn.models.llama import Llama, llama_config

        cfg = llama_config(args.tf_config or "llama3-8b")
        with torch.device("meta"):
            model = Llama(cfg)
        per_gpu = args.tf_batch_per_gpu or 4
    gbatch = per_gpu * world
    opt = FusedAdam(model.parameters(), lr=1e-4, weight_decay=0.01)
    if world == 1 and any(p.is_meta for p in model.parameters()):
        # one GPU holds the whole model whatever the plan: materialise it before planning, so the
        # planner's chain calibration runs the real layers (N > 1: each rank builds its own stage)
        from madnn.parallel.pp import materialize_

        materialize_(model, madnn.device(), getattr(model, "init_weights", None), opt)
    engine, opt = madnn.distribute(model, opt, strategy=args.strategy, checkpointing=args.checkpointing,
                                   global_batch=gbatch,
                                   example_input=torch.zeros(1, seq, dtype=torch.long))
    plan = getattr(engine, "plan", None)
    dp = plan.dp if plan is not None else world
    stages = plan.pp if plan is not None else 1
    replica = rank // stages if stages > 1 else rank
    g = torch.Generator(device="cpu").manual_seed(4321 + replica)
    ids = torch.randint(0, cfg.vocab_size, (gbatch // dp, seq), generator=g).to(madnn.device())

    def step():
        loss = engine.train_step(ids, ids)
        opt.step()
        return loss

    tw = time.perf_counter()
    tuning = 2 * len(getattr(engine, "_lags", [0.0])) if len(getattr(engine, "_lags", [0.0])) > 1 else 0
    for _ in range(max(args.warmup, tuning + 1)):
        step()
    _sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    _sync_all()
    dt = _max_over_ranks(time.perf_counter() - t0)
    lv = float(loss.detach()) if loss is not None else None
    held = _heldout_loss(engine, model, cfg.vocab_size, ids.shape, 98765 + replica, stages, rank)
    ck = sum(bool(c) for c in plan.checkpoint) if plan is not None and plan.checkpoint else 0
    nl = len(plan.checkpoint) if plan is not None and plan.checkpoint else None
    tok = gbatch * seq * args.steps / dt
    return {"metric": TF_METRIC[name], "value": round(tok, 1), "unit": "tokens/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1000.0, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if madnn.device().type == "cuda" else "fp32",
            "data": "synthetic (random tokens, random-init weights)",
            "config": {"model": args.tf_config or name, "global_batch": gbatch, "per_gpu_batch": per_gpu,
                       "seq_len": seq, "parallelism": _parallelism(plan, world), "optimizer": "FusedAdam",
                       "checkpointing": args.checkpointing,
                       "checkpointed_layers": ck, "layers": nl, "peak_mem_gib": _peak_gib(),
                       "warmup_s": round(t0 - tw, 1), "loss": lv, "heldout_loss": held,
                       "ln_vocab": round(math.log(cfg.vocab_size), 4), "plan": _plan_info(plan),
                       "plan_table": plan.table() if plan is not None else None,
                       "samples_per_s": round(gbatch * args.steps / dt, 2)}}


def _peak_gib():
    """This rank's peak allocated device memory (GiB) since the last reset; None on CPU."""
    if not torch.cuda.is_available():
        return None
    return round(torch.cuda.max_memory_allocated() / 2**30, 2)


def _max_over_ranks(dt: float) -> float:
    import madnn

    t = torch.tensor([dt], dtype=torch.float64, device=madnn.device())
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def _release(*objs):
    import gc

    for o in objs:
        del o
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()


def _fail(msg: str, rc: int = 2):
    print(f"bench: error: {msg}", file=sys.stderr, flush=True)
    sys.exit(rc)


def _self_launch(args) -> int:
    """``bench.py --gpus N`` (N > 1) without a launcher: start N ranks here, with the
    ``madnn.launch`` contract (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, teardown of every rank
    at the first failure) -- the reference's one-command ``mpirun -n $nodes`` launch
    (cifar_example/train.sh:14).  This process makes no GPU call: it only counts devices (no HIP
    initialisation on this image), spawns the children (never ``exec``) and returns the exit code
    of the job; rank 0's JSON line reaches stdout through the inherited descriptor."""
    n = args.gpus
    if args.device != "cpu":
        avail = torch.cuda.device_count()
        if avail < n:
            _fail(f"--gpus {n} needs {n} visible devices, this host shows {avail}"
                  f" (HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES')!r},"
                  f" CUDA_VISIBLE_DEVICES={os.environ.get('CUDA_VISIBLE_DEVICES')!r})")
    from madnn.launch import main as launch

    print(f"bench: no launcher environment: starting {n} ranks (madnn.launch)", file=sys.stderr, flush=True)
    return launch(["--nproc", str(n), os.path.abspath(__file__)] + sys.argv[1:])


def _check_ranks(args) -> dict:
    """Every rank checks that the job is what ``--gpus`` says: the process group has exactly N
    ranks and, on GPUs, each rank holds its own existing device (distinct across ranks).  Any
    mismatch exits non-zero with the reason instead of measuring a smaller world."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world != args.gpus:
        _fail(f"--gpus {args.gpus} but the process group has {world} rank(s)")
    import socket

    dev = "cpu"
    if args.device != "cpu":
        if not torch.cuda.is_available():
            _fail(f"--device {args.device}: no GPU visible to rank {dist.get_rank() if dist.is_initialized() else 0}")
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # --backend gloo on GPUs is the one-GPU rehearsal of the N-rank path (RCCL refuses two
        # ranks per device): ranks may share the device there, and the record says so
        rehearsal = args.backend == "gloo"
        if local >= torch.cuda.device_count() and not rehearsal:
            _fail(f"LOCAL_RANK {local} but only {torch.cuda.device_count()} device(s) are visible")
        props = torch.cuda.get_device_properties(torch.cuda.current_device())
        ident = getattr(props, "uuid", None) or getattr(props, "pci_bus_id", None) or torch.cuda.current_device()
        dev = f"{socket.gethostname()}/cuda:{torch.cuda.current_device()}/{ident}"
    devices = [dev]
    if world > 1:
        devices = [None] * world
        dist.all_gather_object(devices, dev)
        if args.device != "cpu" and len(set(devices)) != world and args.backend != "gloo":
            _fail(f"ranks share devices: {devices}")
    out = {"ranks_seen": world, "devices": devices}
    if args.device != "cpu" and len(set(devices)) != world:
        out["shared_devices"] = "gloo rehearsal"
    return out


def main():
    args = parse()
    if args.gpus < 1:
        _fail(f"--gpus {args.gpus}")
    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(_self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        _fail(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={world} rank(s)")
    if not args.no_pg and "RANK" not in os.environ:
        # no launcher: join a world-1 group anyway (same RCCL path as the N-GPU run)
        from madnn.launch import _free_port

        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                          MASTER_PORT=os.environ.get("MASTER_PORT") or str(_free_port()))
    import madnn

    torch.backends.cudnn.benchmark = bool(args.miopen_benchmark)
    madnn.init(device=args.device, backend=args.backend)
    _RANKS.update(_check_ranks(args))
    rank = madnn.get_rank()
    on_gpu = madnn.device().type == "cuda"
    if args.seq_len is None:
        args.seq_len = {"bert-large": 512, "llama3-8b": 4096}.get(args.model, 1024)
    if args.model in TF_METRIC:
        res = bench_transformer(args, world, rank)
        if rank == 0:
            print(res["config"].pop("plan_table") or "", file=sys.stderr)
        _emit(res, rank, args)
        madnn.shutdown()
        return
    res = None
    if args.model in ("all", "resnet50"):
        dt, samples_per_step, config = bench_resnet(args, world, rank)
        dt = _max_over_ranks(dt)
        res = {
            "metric": METRIC,
            "value": round(samples_per_step * args.steps / dt, 2),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1000.0, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic (random ImageNet-shaped images / random tokens, random-init weights)",
            "config": config,
        }
        config["per_gpu_value"] = float(f"{res['value'] / world:.6g}")
        _release()
        if args.std_batch and args.std_batch != config["per_gpu_batch"]:
            # the same measurement at a standard per-GPU batch, so rounds compare like for like
            sargs = argparse.Namespace(**dict(vars(args), batch=args.std_batch))
            sdt, sps_step, sconf = bench_resnet(sargs, world, rank)
            sdt = _max_over_ranks(sdt)
            sval = round(sps_step * args.steps / sdt, 2)
            res["config"]["std_batch"] = {"per_gpu_batch": args.std_batch, "global_batch": sps_step,
                                          "value": sval, "per_gpu_value": float(f"{sval / world:.6g}"),
                                          "ms_per_step": round(sdt / args.steps * 1000.0, 3),
                                          "warmup_s": sconf["warmup_s"], "parallelism": sconf["parallelism"],
                                          **{k: sconf.get(k) for k in ("comm_exposed_ms", "busbw_gbps", "p2p_gbps")}}
            _release()
    if args.model in ("all", "gpt2-medium"):
        if args.model == "all":
            import gc

            gc.collect()
        g = _gpt2_phase(args, world, rank, on_gpu, res)
        if res is None:
            res = {"metric": METRIC, "value": g.get("samples_per_s"), "unit": "samples/s", "n_gpus": world,
                   "steps": g.get("steps", args.steps), "warmup": g.get("warmup", args.warmup),
                   "ms_per_step": g.get("ms_per_step"), "higher_is_better": True, "scaling": "weak",
                   "vs_baseline": None, "dtype": g["dtype"], "data": g["data"],
                   "config": {"model": args.gpt2_config, "global_batch": g.get("global_batch"),
                              "seq_len": args.seq_len, "parallelism": g.get("parallelism")}}
        res["gpt2_pp"] = g
        if "error" in g:
            # peers may be stuck inside the failed phase: no collective teardown.  Only rank 0
            # prints; the others wait for its line (its watchdog fires at the latest after
            # --gpt2-timeout) because a launcher tears the whole job down at the first exit.
            if rank == 0:
                _emit(res, rank, args)
            else:
                time.sleep(args.gpt2_timeout + 60)
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(3)
    _emit(res, rank, args)
    madnn.shutdown()


_RANKS: dict = {}   # ranks_seen / devices of this job (_check_ranks), added to every record


def _emit(res, rank, args):
    if rank == 0:
        line = json.dumps(dict(res, **_RANKS))
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")


def _gpt2_phase(args, world, rank, on_gpu, res):
    """The GPT-2 half as its own failure domain: an exception, or no result within
    ``--gpt2-timeout`` seconds (a hang inside a collective), yields ``{"error": ...}`` and the
    already measured ResNet value is still printed (rank 0's watchdog prints it and ends the
    process if the phase never returns)."""
    import threading

    base = {"model": args.gpt2_config, "n_gpus": world, "scaling": "weak", "dtype": "bf16" if on_gpu else "fp32",
            "data": "synthetic (random tokens, random-init weights)"}
    strategy, stages, par = gpt2_layout(world)
    base["parallelism"] = par
    done = threading.Event()

    def watchdog():
        if done.wait(args.gpt2_timeout):
            return
        out = dict(res or {"metric": METRIC, "value": None, "n_gpus": world})
        out["gpt2_pp"] = dict(base, error=f"timeout: GPT-2 phase did not finish within {args.gpt2_timeout:.0f} s")
        print(f"bench: rank {rank}: GPT-2 phase timed out after {args.gpt2_timeout:.0f} s", file=sys.stderr,
              flush=True)
        _emit(out, rank, args)
        sys.stdout.flush()
        os._exit(3)

    wd = threading.Thread(target=watchdog, daemon=True)
    wd.start()
    fault = os.environ.get("MADNN_BENCH_GPT2_FAULT")
    if fault:  # madnn's fault injection (MADNN_FAULT=rank:step:kind), armed for this phase only
        os.environ["MADNN_FAULT"] = fault
    try:
        dt, steps, gbatch, info = bench_gpt2(args, world, rank)
        dt = _max_over_ranks(dt)
    except Exception as e:  # noqa: BLE001
        done.set()
        print(f"bench: rank {rank}: GPT-2 phase failed: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        return dict(base, error=f"{type(e).__name__}: {str(e)[:300]}")
    done.set()
    sps = gbatch * steps / dt
    return dict(base, **info, samples_per_s=round(sps, 2), tokens_per_s=round(sps * args.seq_len, 1),
                ms_per_step=round(dt / steps * 1000.0, 3))


if __name__ == "__main__":
    main()
