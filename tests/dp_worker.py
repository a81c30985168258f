"""Worker for the multi-process data-parallel tests (gloo, CPU).

Run as ``python tests/dp_worker.py <mode> <outdir>`` with the torch.distributed
env contract set by the launcher under test."""

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402


def make_model():
    torch.manual_seed(1234)
    from zookeeper_amd.nn import QuantDense

    return nn.Sequential(
        nn.Linear(12, 32), nn.Tanh(),
        QuantDense(32, 16, "ste_sign", "ste_sign", "weight_clip"),
        nn.Linear(16, 5),
    )


def data(global_batch=8, steps=3):
    g = torch.Generator().manual_seed(7)
    xs = torch.randn(steps, global_batch, 12, generator=g)
    ys = torch.randint(0, 5, (steps, global_batch), generator=g)
    return xs, ys


def train(rank, world, bucket_mb, check_order=False):
    from zookeeper_amd.core import configure
    from zookeeper_amd.parallel import dist as zdist
    from zookeeper_amd.train import Adam, Trainer

    comm = zdist.CommConfig(check_bucket_order=check_order)
    info = zdist.init("gloo", comm=comm) if world > 1 else zdist.DistInfo()
    spec = Adam()
    configure(spec, {"learning_rate": 0.01})
    model = make_model()
    if rank == 1:  # different init on rank 1: the broadcast must fix it
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    tr = Trainer(model, "sparse_categorical_crossentropy", spec, info, bucket_mb=bucket_mb,
                 first_bucket_mb=0.0005)
    xs, ys = data()
    per = xs.shape[1] // world
    for s in range(xs.shape[0]):
        x = xs[s, rank * per:(rank + 1) * per]
        y = ys[s, rank * per:(rank + 1) * per]
        tr.train_step(x, y)
    return tr


if __name__ == "__main__":
    mode, out = sys.argv[1], sys.argv[2]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if mode == "fail" and rank == 1:
        sys.exit(3)
    if mode == "fail":
        import time

        time.sleep(60)  # would hang; the launcher must terminate us
        sys.exit(0)
    if mode == "hang":
        # rank 1 hangs without ever joining the collective; rank 0's
        # all-reduce must time out (ZK_DIST_TIMEOUT_S) and exit non-zero so
        # the launcher tears the job down instead of waiting forever
        import time

        from zookeeper_amd.parallel import dist as zdist

        zdist.init("gloo")
        if rank == 1:
            time.sleep(600)
            sys.exit(0)
        t = torch.ones(4)
        torch.distributed.all_reduce(t)  # raises after the timeout
        sys.exit(0)
    if mode == "bnsync":
        # BN running statistics drift apart per rank; all_reduce_buffers
        # must leave every rank with the cross-rank mean
        from zookeeper_amd.parallel import dist as zdist
        from zookeeper_amd.parallel.ddp import all_reduce_buffers

        zdist.init("gloo")
        torch.manual_seed(0)
        bn = nn.BatchNorm1d(6)
        bn.train()
        g = torch.Generator().manual_seed(100 + rank)
        for _ in range(3):
            bn(torch.randn(16, 6, generator=g) * (rank + 1) + rank)
        before = {k: v.clone() for k, v in bn.state_dict().items()}
        all_reduce_buffers(bn)
        torch.save({"before": before, "after": bn.state_dict()},
                   os.path.join(out, f"bn{rank}.pt"))
        zdist.shutdown()
        sys.exit(0)
    if mode == "order":
        # the bucket-order check must flag ranks that launch differently
        from zookeeper_amd.parallel import dist as zdist

        tr = train(rank, world, bucket_mb=0.001, check_order=True)
        ok_checks = tr.bucketer.order_checks
        try:
            tr.bucketer.compare_order([0, 1] if rank == 0 else [1, 0])
            flagged = False
        except RuntimeError:
            flagged = True
        torch.save({"checks": ok_checks, "order": tr.bucketer.last_order, "flagged": flagged},
                   os.path.join(out, f"order{rank}.pt"))
        zdist.shutdown()
        sys.exit(0)
    tr = train(rank, world, bucket_mb=0.001)
    torch.save({"params": tr.flat.data.clone(), "buckets": tr.bucketer.num_buckets},
               os.path.join(out, f"rank{rank}.pt"))
