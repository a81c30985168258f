#!/usr/bin/env python
"""Headline benchmark: training throughput (images/sec, whole job) of
BinaryResNet-E18 on ImageNet-shape synthetic data (224×224×3, 1000 classes,
random-init weights), data parallel over RCCL with one process per GPU.

    python bench.py --gpus 1 --steps 30 --warmup 10
    python bench.py --gpus 8                      # spawns 8 ranks itself
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8

``--gpus N`` with N > 1 and no ``WORLD_SIZE`` in the environment starts N
rank processes itself (``zookeeper_amd.parallel.launch.spawn``: subprocesses,
before anything touches the GPU, never exec) and returns their exit code.
Inside a launched job ``WORLD_SIZE`` must equal ``--gpus``: a mismatch is an
error, never a silent 1-GPU run.

A timed step is the complete training step: uint8→bf16 normalisation/flip
of the batch, forward, softmax-CE, backward with bucketed all-reduce on a
comm stream, fused Adam + weight_clip.  ``--data stream`` (default) feeds
the synthetic source through the host input pipeline (native row gather into
pinned slots, side-stream H2D, event hand-off), so the host→device path of
the reference's ``tf.data`` pipeline (examples/larq_experiment.py:126-139) is
inside the timed region; ``--data pool`` cycles a few device-resident
synthetic batches instead.  When the warmup shows the step host-bound (small
``--batch``), zero-grad + forward + loss + backward are replayed as one HIP
graph (``--graph auto``; under DP the all-reduce runs after the replay).
``--steps`` steps are timed between a barrier + ``torch.cuda.synchronize()``
on both sides; the reported time is the MAX over ranks.  Per-step GPU times
(events between consecutive steps) give the median / p10 / p90.  Rank 0
prints one JSON line.

Weak scaling: the per-GPU batch (``--batch``, default 1536) is fixed, the
global batch is ``batch × N``.  1536 images per GPU use a part of the 288 GB
of HBM; smaller batches leave the 14x14 / 7x7 stages latency-bound (1 GPU,
E18, round 2: 41.3k img/s at 512, 43.1k at 768, 44.0k at 1024; round 3:
46.7k at 1024, 47.9k at 1536, 2048 no faster and with multi-second
allocator stalls), and the fixed-size gradient all-reduce is a smaller share
of a longer step.
"""

import argparse
import json
import os
import sys
import time
from typing import Tuple

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# hardware queues for the step's streams (at least 16), before anything initialises HIP
# (zookeeper_amd/parallel/devices.py: with HIP's default 4 the gradient
# all-reduce's stream waits stalled the input copies, ~15 % under DP)
from zookeeper_amd.parallel.devices import configure_hw_queues  # noqa: E402

configure_hw_queues()

METRIC = "images/sec (whole node) BinaryResNet-E18 ImageNet at 1/2/4/8 MI355X"
OTHER_METRIC = "images/sec (whole node) {model} ImageNet-shape training"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1536, help="per-GPU batch")
    ap.add_argument("--model", default="BinaryResNetE18")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--num-classes", type=int, default=1000)
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--data", default="stream", choices=["pool", "stream"],
                    help="pool: device-resident synthetic batches; stream: host pipeline "
                         "(pinned ring + side-stream H2D) inside the timed region")
    ap.add_argument("--pool", type=int, default=4, help="device-resident synthetic batches")
    ap.add_argument("--bucket-mb", type=float, default=10.0)
    ap.add_argument("--graph", default="auto", choices=["0", "1", "auto"],
                    help="replay forward+backward as a HIP graph; auto: when the warmup "
                         "shows the step host-bound")
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="(rehearsal) let several ranks share a GPU (ZK_DIST_BACKEND=gloo)")
    ap.add_argument("--force-dp", action="store_true",
                    help="keep the bucketed all-reduce on with one GPU (1-rank RCCL group): "
                         "the exact multi-GPU step, with its comm timings")
    ap.add_argument("--rt", action="append", default=[], metavar="KEY=VALUE",
                    help="Runtime component option (zookeeper_amd/train/runtime.py), e.g. "
                         "--rt bconv_fp4=False --rt tile_huge=0; recorded in the JSON")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args(argv)


def _native_digest(backend):
    """Source digest embedded in the loaded native library (which kernels ran)."""
    if backend != "hip":
        return None
    from zookeeper_amd.ops import _native

    d = _native.build_digest()
    return d[:16] if d else None


def _percentile(xs, q):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


def self_launch(args) -> int:
    """Start ``--gpus`` ranks of this script (subprocesses; the parent never
    initialises the GPU) and return the first non-zero exit code."""
    from zookeeper_amd.parallel.launch import spawn

    if not args.allow_shared_gpu:
        # env + sysfs only: the parent must never initialise the HIP runtime
        from zookeeper_amd.parallel.devices import visible_gpu_count

        have = visible_gpu_count()
        if have and have < args.gpus:
            print(f"error: --gpus {args.gpus} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    return spawn([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], args.gpus)


def main() -> int:
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args)
    if world_env != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        return 2

    import torch

    from zookeeper_amd import ComponentField, Field, component, configure
    from zookeeper_amd.core.component import base_getattr
    from zookeeper_amd.data import (DeviceLoader, Dataset, ImageNetPreprocessing, Preprocessing,
                                    SyntheticImageNet, make_device_pool_batches)
    from zookeeper_amd import models
    from zookeeper_amd.parallel import dist as zdist
    from zookeeper_amd.train import Adam, OptimizerSpec, Trainer

    from zookeeper_amd.core.utils import parse_value_from_string
    from zookeeper_amd.train.runtime import Runtime

    runtime = Runtime()
    rt_conf = {}
    for kv in args.rt:
        k, _, v = kv.partition("=")
        rt_conf[k] = parse_value_from_string(v)
    rt_conf.setdefault("graph", {"0": "off", "1": "on", "auto": "auto"}[args.graph])
    if args.force_dp:
        rt_conf["force_dp"] = True
    configure(runtime, rt_conf)
    runtime.apply()
    info = zdist.init(single_group=runtime.force_dp, comm=runtime.comm_config())
    if info.world != args.gpus:
        print(f"error: --gpus {args.gpus} but the job has {info.world} rank(s)", file=sys.stderr)
        return 2
    if (info.world > 1 and torch.cuda.is_available() and not args.allow_shared_gpu
            and torch.cuda.device_count() < info.world):
        print(f"error: {info.world} ranks but {torch.cuda.device_count()} GPU(s)", file=sys.stderr)
        return 2
    S = args.image_size

    @component
    class BenchConfig:
        dataset: Dataset = ComponentField(SyntheticImageNet)
        input_shape: Tuple[int, int, int] = Field((S, S, 3))
        preprocessing: Preprocessing = ComponentField(ImageNetPreprocessing)
        model: torch.nn.Module = ComponentField(getattr(models, args.model))
        optimizer: OptimizerSpec = ComponentField(Adam)
        learning_rate: float = Field(2e-3)

    cfg = BenchConfig()
    configure(cfg, {"dataset.image_shape": (S, S, 3), "dataset.num_classes": args.num_classes,
                    "model.backend": args.backend})
    model = cfg.model
    backend = base_getattr(cfg, "model").resolved_backend()
    torch.manual_seed(1234)
    dp = info.world > 1 or runtime.force_dp
    trainer = Trainer(model, "sparse_categorical_crossentropy", base_getattr(cfg, "optimizer"),
                      info, bucket_mb=args.bucket_mb, graph=runtime.trainer_graph(),
                      graph_warmup=max(1, min(3, args.warmup - 1)),  # capture inside the warmup
                      comm_timing=dp and runtime.comm_timing and torch.cuda.is_available(),
                      force_dp=runtime.force_dp)
    prep = cfg.preprocessing
    loader = None
    if args.data == "stream":
        src, _ = cfg.dataset.train()
        loader = DeviceLoader(src, args.batch, info.device, shuffle=True, seed=0,
                              rank=info.rank, world=info.world, slots=4,
                              transform=(prep.device_transform(training=True)
                                         if runtime.loader_preprocess else None))
        it = iter(loader)
        next_batch = lambda i: next(it)  # noqa: E731
    else:
        pool = make_device_pool_batches(args.pool, args.batch, (S, S, 3), args.num_classes,
                                        info.device, seed=info.rank)
        next_batch = lambda i: pool[i % len(pool)]  # noqa: E731

    cuda = torch.cuda.is_available()
    sync = torch.cuda.synchronize if cuda else (lambda: None)

    def step(i):
        x, y = prep(next_batch(i), training=True)
        return trainer.train_step(x, y)

    t_w = time.perf_counter()
    for i in range(args.warmup):
        loss, _ = step(i)
        if info.is_main and (i == 0 or (i + 1) % 10 == 0):
            sync()
            print(f"[bench] warmup {i + 1}/{args.warmup} loss={loss.item():.4f} "
                  f"t={time.perf_counter() - t_w:.1f}s", file=sys.stderr, flush=True)
    sync()
    trainer.bucketer.pop_timings()  # discard warmup comm timings
    zdist.barrier()
    sync()
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)] if cuda else []
    mem0 = torch.cuda.memory_stats(info.device) if cuda else {}
    host_t = []  # host time per step (enqueue, including any blocking call)
    t0 = time.perf_counter()
    if marks:
        marks[0].record()
    for i in range(args.steps):
        th = time.perf_counter()
        loss, _ = step(args.warmup + i)
        if marks:
            marks[i + 1].record()
        host_t.append(time.perf_counter() - th)
        if info.is_main and (i + 1) % 50 == 0:
            print(f"[bench] step {i + 1}/{args.steps}", file=sys.stderr, flush=True)
    t_enq = time.perf_counter() - t0  # host time to enqueue (no sync yet)
    sync()
    zdist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = zdist.all_reduce_max(elapsed)
    final_loss = float(loss.item())
    step_ms = [marks[i].elapsed_time(marks[i + 1]) for i in range(args.steps)] if marks else []
    mem1 = torch.cuda.memory_stats(info.device) if cuda else {}
    # allocator activity inside the timed region (device mallocs / frees /
    # OOM retries would stall the host: reported so an outlier step has a cause)
    alloc_delta = {k: mem1.get(k, 0) - mem0.get(k, 0)
                   for k in ("num_device_alloc", "num_device_free", "num_alloc_retries")}
    if info.is_main and step_ms:
        worst = max(range(len(step_ms)), key=lambda i: step_ms[i])
        hw = max(range(len(host_t)), key=lambda i: host_t[i])
        print(f"[bench] slowest step {worst}: GPU {step_ms[worst]:.2f} ms; slowest host step "
              f"{hw}: {1e3 * host_t[hw]:.2f} ms; allocator in timed region {alloc_delta}; "
              f"peak allocated {torch.cuda.max_memory_allocated(info.device) / 2**30:.1f} GiB",
              file=sys.stderr, flush=True)
    comm = trainer.bucketer.pop_timings()
    if loader is not None:
        loader.close()

    ms = 1000.0 * elapsed / args.steps
    if info.is_main and trainer.graph_probe is not None:
        th, tg = trainer.graph_probe
        print(f"[bench] graph probe: host {1e3 * th:.2f} ms, GPU {1e3 * tg:.2f} ms -> "
              f"{'graph' if trainer.graph else 'eager'}", file=sys.stderr, flush=True)
    if info.is_main:
        # enqueue ~ total: host-bound; enqueue << total: the GPU is the limit
        print(f"[bench] host enqueue {1000.0 * t_enq / args.steps:.2f} ms/step of {ms:.2f}",
              file=sys.stderr, flush=True)
    global_batch = args.batch * info.world
    value = global_batch * args.steps / elapsed
    r3 = lambda v: None if v is None else round(v, 3)  # noqa: E731
    data_desc = (f"synthetic (ImageNet-shape uint8 {S}x{S}x3, {args.num_classes} classes, "
                 + ("device-resident pool" if args.data == "pool" else
                    "host source streamed: native gather into pinned slots + side-stream H2D")
                 + "; random-init weights)")
    # the headline metric string only for the headline configuration on its
    # real transport: one GPU per rank, RCCL between them
    rehearsal = args.allow_shared_gpu or (info.world > 1 and info.backend != "nccl") \
        or not torch.cuda.is_available()
    headline = (args.model == "BinaryResNetE18" and S == 224 and args.num_classes == 1000)
    metric = METRIC if headline else OTHER_METRIC.format(model=args.model)
    if rehearsal:
        metric = f"rehearsal ({info.backend if info.world > 1 else 'cpu'}, not a measurement): " \
            + metric
    out = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": info.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "ms_per_step_median": r3(_percentile(step_ms, 0.5)),
        "ms_per_step_p10": r3(_percentile(step_ms, 0.1)),
        "ms_per_step_p90": r3(_percentile(step_ms, 0.9)),
        "ms_per_step_max": r3(max(step_ms)) if step_ms else None,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": data_desc,
        "config": {
            "model": args.model,
            "global_batch": global_batch,
            "per_gpu_batch": args.batch,
            "seq_len": None,
            "image_shape": [S, S, 3],
            "parallelism": f"dp{info.world}",
            "backend": backend,
            "native_digest": _native_digest(backend),
            "optimizer": "adam+weight_clip (fused)",
            "hip_graph": trainer.graph,
            "data_path": args.data,
            "buckets": trainer.bucketer.num_buckets if trainer.bucketer.enabled else 0,
            "dist_backend": info.backend,
            "comm": {"cpu_affinity_cpus": len(info.cpus) if info.cpus else None,
                     "rccl_env": info.rccl_env,
                     "rccl_high_priority": bool(runtime.comm_high_priority and dp),
                     "bucket_mb": args.bucket_mb,
                     "bucket_sizes_mb": [round((hi - lo) * 4 / 2**20, 2)
                                         for lo, hi in trainer.bucketer.ranges],
                     "bucket_order_checks": trainer.bucketer.order_checks,
                     "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")},
            "runtime": runtime.as_dict(),
            "final_loss": round(final_loss, 4),
        },
    }
    if comm:
        out["comm"] = {
            "comm_ms_median": r3(_percentile([c["comm_ms"] for c in comm], 0.5)),
            "bucket_sum_ms_median": r3(_percentile([c["bucket_sum_ms"] for c in comm], 0.5)),
            "exposed_ms_median": r3(_percentile([c["exposed_ms"] for c in comm], 0.5)),
            "exposed_ms_max": r3(max(c["exposed_ms"] for c in comm)),
        }
    if info.is_main:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    zdist.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
