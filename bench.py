#!/usr/bin/env python
"""Headline benchmark: training throughput (images/sec, whole job) of
BinaryResNet-E18 on ImageNet-shape synthetic data (224×224×3, 1000 classes,
random-init weights), data parallel over RCCL with one process per GPU.

    python bench.py --gpus 1 --steps 30 --warmup 10
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
        --master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8

A timed step is the complete training step: uint8→bf16 normalisation/flip
of the batch, forward, softmax-CE, backward with bucketed all-reduce, fused
Adam + weight_clip.  Input batches come from a device-resident pool of
synthetic batches (no host work per step).  On one GPU, when the warmup
shows the step host-bound (small ``--batch``), zero-grad + forward + loss +
backward are replayed as one HIP graph (``--graph auto``); the optimizer
still runs every step.  ``--steps`` steps are timed
between a barrier + ``torch.cuda.synchronize()`` on both sides; the reported
time is the MAX over ranks.  Rank 0 prints one JSON line.

Weak scaling: the per-GPU batch (``--batch``, default 512) is fixed, the
global batch is ``batch × N``.  512 images per GPU use a few GB of the 288 GB
of HBM; at 256 the small late-stage layers leave the step partly
latency-bound (1 GPU: 36.7k img/s at 256, 39.0k at 384, 40.1k at 512).
"""

import argparse
import json
import os
import sys
import time
from typing import Tuple

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

METRIC = "images/sec (whole node) BinaryResNet-E18 ImageNet at 1/2/4/8 MI355X"
OTHER_METRIC = "images/sec (whole node) {model} ImageNet-shape training"


def parse():
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=512, help="per-GPU batch")
    ap.add_argument("--model", default="BinaryResNetE18")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    ap.add_argument("--pool", type=int, default=4, help="device-resident synthetic batches")
    ap.add_argument("--bucket-mb", type=float, default=25.0)
    ap.add_argument("--graph", default="auto", choices=["0", "1", "auto"],
                    help="replay forward+backward as a HIP graph (1 GPU; eager when distributed); "
                         "auto: when the warmup shows the step host-bound")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def main() -> int:
    args = parse()
    import torch

    from zookeeper_amd import ComponentField, Field, component, configure
    from zookeeper_amd.core.component import base_getattr
    from zookeeper_amd.data import (Dataset, ImageNetPreprocessing, Preprocessing,
                                    SyntheticImageNet, make_device_pool_batches)
    from zookeeper_amd import models
    from zookeeper_amd.parallel import dist as zdist
    from zookeeper_amd.train import Adam, OptimizerSpec, Trainer

    info = zdist.init()
    if info.world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={info.world}", file=sys.stderr)

    @component
    class BenchConfig:
        dataset: Dataset = ComponentField(SyntheticImageNet)
        input_shape: Tuple[int, int, int] = Field((224, 224, 3))
        preprocessing: Preprocessing = ComponentField(ImageNetPreprocessing)
        model: torch.nn.Module = ComponentField(getattr(models, args.model))
        optimizer: OptimizerSpec = ComponentField(Adam)
        learning_rate: float = Field(2e-3)

    cfg = BenchConfig()
    configure(cfg, {"model.backend": args.backend})
    model = cfg.model
    backend = base_getattr(cfg, "model").resolved_backend()
    torch.manual_seed(1234)
    trainer = Trainer(model, "sparse_categorical_crossentropy", base_getattr(cfg, "optimizer"),
                      info, bucket_mb=args.bucket_mb,
                      graph="auto" if args.graph == "auto" else args.graph == "1",
                      graph_warmup=max(1, min(3, args.warmup - 1)))  # capture inside the warmup
    pool = make_device_pool_batches(args.pool, args.batch, (224, 224, 3), 1000, info.device,
                                    seed=info.rank)
    prep = cfg.preprocessing

    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)

    def step(i):
        x, y = prep(pool[i % len(pool)], training=True)
        return trainer.train_step(x, y)

    # ZK_MAIN_PRIORITY (experiment): run the step on a compute stream of that
    # HIP priority (negative = above the side stream of the weight gradients)
    main_prio = os.environ.get("ZK_MAIN_PRIORITY")
    if main_prio and torch.cuda.is_available():
        main_stream = torch.cuda.Stream(priority=int(main_prio))
        main_stream.wait_stream(torch.cuda.current_stream())
        torch.cuda.set_stream(main_stream)

    t_w = time.perf_counter()
    for i in range(args.warmup):
        loss, _ = step(i)
        if info.is_main and (i == 0 or (i + 1) % 10 == 0):
            sync()
            print(f"[bench] warmup {i + 1}/{args.warmup} loss={loss.item():.4f} "
                  f"t={time.perf_counter() - t_w:.1f}s", file=sys.stderr, flush=True)
    zdist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss, _ = step(args.warmup + i)
        if info.is_main and (i + 1) % 50 == 0:
            print(f"[bench] step {i + 1}/{args.steps}", file=sys.stderr, flush=True)
    t_enq = time.perf_counter() - t0  # host time to enqueue (no sync yet)
    sync()
    zdist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = zdist.all_reduce_max(elapsed)
    final_loss = float(loss.item())

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
    out = {
        "metric": METRIC if args.model == "BinaryResNetE18" else OTHER_METRIC.format(model=args.model),
        "value": round(value, 2),
        "unit": "images/sec",
        "n_gpus": info.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (ImageNet-shape uint8 224x224x3, 1000 classes, device-resident pool; random-init weights)",
        "config": {
            "model": args.model,
            "global_batch": global_batch,
            "per_gpu_batch": args.batch,
            "seq_len": None,
            "image_shape": [224, 224, 3],
            "parallelism": f"dp{info.world}",
            "backend": backend,
            "optimizer": "adam+weight_clip (fused)",
            "hip_graph": trainer.graph,
            "final_loss": round(final_loss, 4),
        },
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
