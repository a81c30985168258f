"""Diagnostic: is a wait recorded on a stream that carries no work of its own
honoured by an event recorded on that stream afterwards?

The gloo stager's chain: side stream (weight gradient) --event--> comm stream
(waits only) --event recorded on comm--> copy stream in a worker thread (D2H of
the gradient).  ``direct=1``: the copy stream waits on the side event itself.

    python scripts/diag_wait_chain.py [iters] [comm_priority] [direct]
"""
import queue
import sys
import threading

import torch


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    prio = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    direct = len(sys.argv) > 3 and sys.argv[3] == "1"
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    comm = torch.cuda.Stream(dev, priority=prio)
    a = torch.randn(2048, 2048, device=dev)
    x = torch.zeros(1 << 22, device=dev)
    host = torch.empty(1 << 22, pin_memory=True)
    q, res = queue.Queue(), queue.Queue()

    def worker():
        copy = torch.cuda.Stream(dev)
        while True:
            item = q.get()
            if item is None:
                return
            k, evs = item
            for ev in evs:
                copy.wait_event(ev)
            with torch.cuda.stream(copy):
                host.copy_(x, non_blocking=False)
            res.put(int((host != float(k)).sum()))

    th = threading.Thread(target=worker, daemon=True)
    th.start()
    bad = 0
    for k in range(1, iters + 1):
        cur = torch.cuda.current_stream()
        x.zero_()
        start = torch.cuda.Event()
        start.record(cur)
        side.wait_event(start)
        with torch.cuda.stream(side):
            b = a
            for _ in range(12):
                b = b @ a
                b = b / b.abs().max()
            x.fill_(float(k))
            x.add_(b[0, 0] * 0)
            done = torch.cuda.Event()
            done.record(side)
        ready = torch.cuda.Event()
        ready.record(cur)
        comm.wait_event(ready)
        comm.wait_event(done)
        ready2 = torch.cuda.Event()
        ready2.record(comm)
        q.put((k, [ready, done] if direct else [ready2]))
        n = res.get()
        bad += n > 0
        cur.wait_event(done)
        torch.cuda.synchronize()
    q.put(None)
    th.join()
    print(f"wait chain prio={prio} direct={direct}: {bad}/{iters} copies saw stale data",
          flush=True)


if __name__ == "__main__":
    main()
