"""Local multi-process launcher (one process per GPU).

``python train.py TrainImageNet --nproc 8 key=value ...`` re-runs the same
command line in ``nproc`` child processes with the ``torch.distributed`` env
contract set (``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``MASTER_ADDR``,
``MASTER_PORT``; ``HSA_ENABLE_IPC_MODE_LEGACY=0`` for RCCL's dmabuf IPC) and
supervises them:

* a rank that exits non-zero makes the launcher terminate the others and
  return that exit code (fail-fast instead of hanging in a collective);
* SIGINT/SIGTERM are forwarded to the children.

The parent never initialises the GPU (children are started with
``subprocess``, never ``exec``), which is a hard requirement on this pool.
"""

from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _strip_option(argv: Sequence[str], name: str) -> List[str]:
    out, skip = [], False
    for i, a in enumerate(argv):
        if skip:
            skip = False
            continue
        if a == name:
            skip = True
            continue
        if a.startswith(name + "="):
            continue
        out.append(a)
    return out


def spawn(argv: Sequence[str], nproc: int, env: Optional[Dict[str, str]] = None,
          master_port: Optional[int] = None, poll_s: float = 0.2,
          log_dir: Optional[str] = None) -> int:
    """Run ``argv`` as ``nproc`` ranks; return the first non-zero exit code."""
    base = dict(os.environ if env is None else env)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    base["MASTER_ADDR"] = "127.0.0.1"
    base["MASTER_PORT"] = str(master_port or free_port())
    base["WORLD_SIZE"] = str(nproc)
    base["LOCAL_WORLD_SIZE"] = str(nproc)
    # CPU ranks (gloo) would each start one OpenMP thread per core
    base.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // nproc)))
    procs: List[subprocess.Popen] = []
    files = []
    for r in range(nproc):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        out = None
        if log_dir is not None:
            os.makedirs(log_dir, exist_ok=True)
            out = open(os.path.join(log_dir, f"rank{r}.log"), "w")
            files.append(out)
        procs.append(subprocess.Popen(list(argv), env=e, stdout=out,
                                      stderr=subprocess.STDOUT if out else None))

    def forward(sig, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(sig)

    old = {s: signal.signal(s, forward) for s in (signal.SIGINT, signal.SIGTERM)}
    code = 0
    try:
        alive = set(range(nproc))
        while alive:
            for r in list(alive):
                rc = procs[r].poll()
                if rc is None:
                    continue
                alive.discard(r)
                if rc != 0 and code == 0:
                    code = rc
                    print(f"[launch] rank {r} exited with code {rc}; terminating the others",
                          file=sys.stderr)
                    for p in procs:
                        if p.poll() is None:
                            p.terminate()
            time.sleep(poll_s)
        # give terminated ranks a moment, then kill stragglers
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    finally:
        for s, h in old.items():
            # None: the previous handler was installed outside Python (e.g. by
            # a profiler's preloaded library) and cannot be reinstated from here
            signal.signal(s, h if h is not None else signal.SIG_DFL)
        for f in files:
            f.close()
    return code


def maybe_relaunch(nproc: int) -> Optional[int]:
    """Called from a task command with ``--nproc``: if this process is not
    already a rank of a job, spawn the ranks and return their exit code."""
    if "RANK" in os.environ and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        return None  # we are a worker already
    argv = _strip_option(sys.argv, "--nproc")
    return spawn([sys.executable, *argv], nproc)
