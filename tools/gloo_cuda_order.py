"""Does ``torch.distributed`` gloo order its CUDA staging by stream events?

Two ranks share the GPU.  Each step: X = rank+1 (64 MiB) on the compute
stream; a comm stream waits on it and issues ``all_reduce(X, async_op=True)``;
``work.wait()`` under the comm stream; the compute stream waits on the comm
stream and immediately clones X.  Every element of the clone must be 3.  A
smaller value means the compute stream ran before gloo's host→device copy of
the result landed, i.e. ``wait()`` did not order the caller's stream.

    python -m tools.gloo_cuda_order          # launches 2 ranks
"""

import os
import sys

import torch


def worker():
    import torch.distributed as dist

    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo", rank=rank, world_size=2)
    torch.cuda.set_device(0)
    comm = torch.cuda.Stream()
    flat = torch.empty(48 * 2**20, device="cuda")
    parts = flat.chunk(6)  # several collectives outstanding, like gradient buckets
    bad = 0
    for it in range(20):
        flat.zero_()
        works = []
        for p in parts:
            p.add_(rank + 1)
            big = torch.randn(2048, 2048, device="cuda")
            for _ in range(3):  # queue some compute so the streams overlap
                big = big @ big
            ev = torch.cuda.Event()
            ev.record()
            comm.wait_event(ev)
            with torch.cuda.stream(comm):
                works.append(dist.all_reduce(p, async_op=True))
        with torch.cuda.stream(comm):
            for w in works:
                w.wait()
        torch.cuda.current_stream().wait_stream(comm)
        y = flat.clone()
        flat.zero_()  # the next step's zero_grad
        torch.cuda.synchronize()
        n = int((y != 3).sum()) + int((flat != 0).sum())
        bad += n > 0
        if n:
            print(f"rank {rank} iter {it}: {n} stale elements (min {float(y.min())})", flush=True)
    print(f"rank {rank}: {bad}/20 iterations saw stale results", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    if "RANK" in os.environ:
        worker()
    else:
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from zookeeper_amd.parallel.launch import spawn

        sys.exit(spawn([sys.executable, os.path.abspath(__file__)], 2))
