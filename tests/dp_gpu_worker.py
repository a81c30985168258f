"""Worker for the data-parallel GPU test: two ranks share the box's GPU and
talk over gloo (RCCL needs one GPU per rank), so the GPU training path --
HIP kernels writing gradients straight into the flat buffer, post-accumulate
hooks and direct-grad readiness driving the bucketed all-reduce, initial
broadcast -- runs multi-rank.

    python tests/dp_gpu_worker.py <same|split> <outdir>

Environment (test knobs of this worker only): ``ZK_TEST_SIDE=0|1``
(side-stream weight gradients, ``runtime.wgrad_side_stream``),
``ZK_TEST_GRAPH=0|1`` (HIP-graph replay under DP), ``ZK_TEST_FORCE_DP=1``
(one rank, but a 1-rank process group of ``ZK_TEST_BACKEND`` -- ``nccl`` is
RCCL -- with the bucketed all-reduce forced on: the exact multi-GPU path on
the box's one GPU).  The bucketer never
synchronises the host: ordering is carried by events alone
(compute → comm stream at bucket-ready, comm → compute before the optimizer).

``same``: every rank trains on the same batches, so the averaged gradients
equal a single process's and the result must match a world-size-1 run
(``world=1`` when launched without the env contract).  ``split``: disjoint
batches; ranks must stay bit-identical.

SGD, not Adam: Adam's first steps are sign(g) * lr, and in a binary network
a weight or activation landing next to zero flips a sign, so fp32-atomics
noise (1e-7, see tools/grad_determinism.py) would make any two runs --
even two single-process ones -- diverge chaotically.  SGD keeps the updates
proportional to the gradients, so runs agree to rounding."""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def run(mode: str, out: str) -> None:
    from zookeeper_amd.core import configure
    from zookeeper_amd.models.binary_resnet import BinaryResNetE
    from zookeeper_amd.parallel import dist as zdist
    from zookeeper_amd.train import SGD, Trainer

    from zookeeper_amd.ops.options import set_options

    world = int(os.environ.get("WORLD_SIZE", "1"))
    force = os.environ.get("ZK_TEST_FORCE_DP", "0") == "1"
    backend = os.environ.get("ZK_TEST_BACKEND", "gloo")
    set_options(wgrad_side_stream=os.environ.get("ZK_TEST_SIDE", "1") == "1")
    # ZK_TEST_RT="key=value,...": further kernel options (diagnostics)
    for kv in filter(None, os.environ.get("ZK_TEST_RT", "").split(",")):
        k, v = kv.split("=")
        set_options(**{k: (v.lower() in ("1", "true")) if v.lower() in ("0", "1", "true", "false")
                       else int(v)})
    # ZK_TEST_CHECK_ORDER=1: every step compares the launched bucket order
    # across ranks (runtime.check_bucket_order)
    comm = zdist.CommConfig(check_bucket_order=os.environ.get("ZK_TEST_CHECK_ORDER", "0") == "1",
                            backend=os.environ.get("ZK_TEST_COMM", "auto"),
                            high_priority=os.environ.get("ZK_TEST_COMM_PRIO", "0") == "1",
                            cpu_affinity=os.environ.get("ZK_TEST_AFFINITY", "1") == "1")
    if world > 1 or force:
        info = zdist.init(backend, single_group=force, comm=comm)
    else:
        info = zdist.init(comm=comm)
    torch.manual_seed(1234)
    model = BinaryResNetE((64, 64, 3), 10, 18, backend="hip")
    if info.rank == 1:  # different init on rank 1: the broadcast must fix it
        with torch.no_grad():
            for p in model.parameters():
                p.add_(0.5)
    spec = SGD()
    configure(spec, {"learning_rate": 1e-2})
    # ZK_TEST_GRAPH=1: forward+backward replayed as a HIP graph (the
    # all-reduce issued on the comm stream after each replay)
    graph = os.environ.get("ZK_TEST_GRAPH", "0") == "1"
    tr = Trainer(model, "sparse_categorical_crossentropy", spec, info, bucket_mb=2.0,
                 first_bucket_mb=0.25, graph=graph, graph_warmup=1,
                 comm_timing=world > 1 or force, force_dp=force)
    init = tr.flat.data.detach().cpu().clone()  # after the initial broadcast
    g = torch.Generator().manual_seed(99)
    steps, per = int(os.environ.get("ZK_TEST_STEPS", "2")), 4
    # the same tensors for every world size (at most 2 ranks)
    xs = torch.randn(steps, 2 * per, 3, 64, 64, generator=g)
    ys = torch.randint(0, 10, (steps, 2 * per), generator=g)
    # ZK_TEST_ABORT_AFTER=k: after step k, mark the native communicator as
    # failed (what the watchdog does on a hung collective); the next step must
    # raise before replaying a graph that holds the aborted communicator's
    # collectives
    abort_after = int(os.environ.get("ZK_TEST_ABORT_AFTER", "-1"))
    replays = [0]
    abort = {}
    for s in range(steps):
        lo = 0 if mode == "same" else info.rank * per
        x = xs[s, lo:lo + per].to(info.device, torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = ys[s, lo:lo + per].to(info.device)
        if s == abort_after + 1 and abort_after >= 0:
            torch.cuda.synchronize()
            native = tr.bucketer.native
            assert native is not None and tr._graph is not None
            real = tr._graph.replay

            def counted():
                replays[0] += 1
                real()

            tr._graph.replay = counted
            native._failed = "injected failure"
            try:
                tr.train_step(x, y)
                abort = {"raised": False}
            except RuntimeError as e:
                abort = {"raised": "injected failure" in str(e)}
            abort["replays"] = replays[0]
            break
        loss, _ = tr.train_step(x, y)
    torch.cuda.synchronize()
    if abort:
        torch.save(abort, os.path.join(out, "abort.pt"))
        zdist.shutdown()
        return
    timings = tr.bucketer.pop_timings()
    torch.save({"params": tr.flat.data.cpu(), "init": init, "loss": float(loss),
                "buckets": tr.bucketer.num_buckets, "graph": tr.graph,
                "comm_steps": len(timings), "timings": timings,
                "backend": info.backend, "bucketer": tr.bucketer.enabled,
                "slots": [(sl.name, sl.offset, sl.numel) for sl in tr.flat.slots],
                "ranges": list(tr.bucketer.ranges),
                "order_checks": tr.bucketer.order_checks,
                "native": tr.bucketer.native is not None,
                "last_order": list(tr.bucketer.last_order)},
               os.path.join(out, f"{mode}_w{world}{'dp' if force else ''}_r{info.rank}.pt"))
    zdist.shutdown()


if __name__ == "__main__":
    run(sys.argv[1], sys.argv[2])
