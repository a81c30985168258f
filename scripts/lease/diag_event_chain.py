"""Diagnostic: is a transitive event chain side -> compute -> comm honoured?

The side stream runs a long kernel chain and then writes ``x``; the compute
stream waits for the side stream's event and records ``ready``; a
(high-priority) comm stream waits for ``ready`` and copies ``x`` to pinned
host memory.  Every copy must see the side stream's final value.

    python scripts/diag_event_chain.py [iters] [comm_priority] [direct]
"""
import sys

import torch


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    prio = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    direct = len(sys.argv) > 3 and sys.argv[3] == "1"
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev, priority=0)
    comm = torch.cuda.Stream(dev, priority=prio)
    a = torch.randn(2048, 2048, device=dev)
    x = torch.zeros(1 << 20, device=dev)
    host = torch.empty(1 << 20, pin_memory=True)
    bad = 0
    for k in range(1, iters + 1):
        cur = torch.cuda.current_stream()
        start = torch.cuda.Event()
        start.record(cur)
        side.wait_event(start)
        with torch.cuda.stream(side):
            b = a
            for _ in range(8):
                b = b @ a
                b = b / b.abs().max()
            x.fill_(float(k))
            x.add_(b[0, 0] * 0)
            done = torch.cuda.Event()
            done.record(side)
        cur.wait_event(done)
        ready = torch.cuda.Event()
        ready.record(cur)
        comm.wait_event(ready)
        if direct:
            comm.wait_event(done)
        with torch.cuda.stream(comm):
            host.copy_(x, non_blocking=True)
            fin = torch.cuda.Event()
            fin.record(comm)
        fin.synchronize()
        if not bool((host == float(k)).all()):
            bad += 1
        cur.wait_stream(comm)
    torch.cuda.synchronize()
    print(f"event chain prio={prio} direct={direct}: {bad}/{iters} copies saw stale data",
          flush=True)


if __name__ == "__main__":
    main()
