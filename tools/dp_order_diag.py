"""Data-parallel ordering diagnostics on one GPU (gloo ranks sharing it):
runs ``tests/dp_gpu_worker.py same`` as 1 and 2 ranks under several
settings and prints the relative parameter error vs the single-process run
(and the noise between two single-process runs).

    python -m tools.dp_order_diag
"""

import itertools
import os
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dp_gpu_worker.py")


def run(out, nproc, **env):
    from zookeeper_amd.parallel.launch import spawn

    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4", **env)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    if nproc == 1:
        return subprocess.run([sys.executable, WORKER, "same", out], env=e, timeout=240).returncode
    return spawn([sys.executable, WORKER, "same", out], nproc, env=e)


def load(d, w, r=0):
    return torch.load(os.path.join(d, f"same_w{w}_r{r}.pt"), weights_only=True)


def rel(a, b, ref):
    upd = (ref["params"] - ref["init"]).norm().item()
    return (a["params"] - b["params"]).norm().item() / upd


def main():
    combos = [("2", "1", "0"), ("2", "1", "0"), ("2", "0", "0"), ("1", "1", "0")]
    for steps, side, hs in combos:
        env = dict(ZK_TEST_STEPS=steps, ZK_TEST_SIDE=side, ZK_COMM_HOST_SYNC=hs)
        with tempfile.TemporaryDirectory() as d1, tempfile.TemporaryDirectory() as d2:
            assert run(d1, 1, **env) == 0
            assert run(d2, 1, **env) == 0
            noise = rel(load(d1, 1), load(d2, 1), load(d1, 1))
            assert run(d1, 2, **env) == 0
            err = rel(load(d1, 2), load(d1, 1), load(d1, 1))
            print(f"steps={steps} side={side} host_sync={hs}: 2-rank err {err:.3e}  "
                  f"1-rank noise {noise:.3e}", flush=True)
            if err > 10 * max(noise, 1e-7):
                a, ref = load(d1, 2), load(d1, 1)
                upd = ref["params"] - ref["init"]
                rows = []
                for name, off, n in a["slots"]:
                    d = (a["params"][off:off + n] - ref["params"][off:off + n]).norm().item()
                    u = upd[off:off + n].norm().item()
                    bk = next(i for i, (lo, hi) in enumerate(a["ranges"]) if lo <= off < hi)
                    rows.append((d / max(u, 1e-30), d, name, bk))
                rows.sort(reverse=True)
                for r in rows[:8]:
                    print(f"    rel {r[0]:.3e} abs {r[1]:.3e} bucket {r[3]} {r[2]}", flush=True)
                print("    buckets:", a["ranges"], flush=True)


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    main()
