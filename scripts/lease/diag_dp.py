"""Diagnostic: which parameter slots differ between data-parallel worker runs
(tests/dp_gpu_worker.py), e.g. world 1 vs world 2 in deterministic mode.

    python scripts/diag_dp.py <outdir> [side] [rt]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests", "gpu"))
sys.path.insert(0, ROOT)

from test_dp_gpu import _run  # noqa: E402


def diff(a, b, tag):
    pa, pb = a["params"], b["params"]
    print(f"== {tag}: equal={torch.equal(pa, pb)}", flush=True)
    if os.environ.get("DIAG_BRIEF"):
        return
    for name, off, n in a["slots"]:
        x, y = pa[off:off + n], pb[off:off + n]
        if not torch.equal(x, y):
            d = (x - y).abs()
            print(f"  {name} off={off} n={n} mismatched={(d > 0).sum().item()} "
                  f"max={d.max().item():.3e}", flush=True)


def main():
    out = sys.argv[1]
    side = sys.argv[2] if len(sys.argv) > 2 else "1"
    rt = sys.argv[3] if len(sys.argv) > 3 else "deterministic=1"
    os.makedirs(out, exist_ok=True)
    reps = int(os.environ.get("DIAG_REPS", "1"))
    if os.environ.get("DIAG_BURN"):
        # world-1 runs under a concurrent GPU load vs one without
        import subprocess
        d = os.path.join(out, "ref")
        os.makedirs(d, exist_ok=True)
        assert _run("same", d, 1, side, "0", rt=rt) == 0
        ref = torch.load(os.path.join(d, "same_w1_r0.pt"), weights_only=True)
        burn = subprocess.Popen([sys.executable, os.path.join(ROOT, "scripts", "lease", "gpu_burn.py"),
                                 str(8 * reps + 20)])
        try:
            for i in range(reps):
                d = os.path.join(out, f"u{i}")
                os.makedirs(d, exist_ok=True)
                assert _run("same", d, 1, side, "0", rt=rt) == 0
                diff(ref, torch.load(os.path.join(d, "same_w1_r0.pt"), weights_only=True),
                     f"w1 vs w1 under load #{i}")
        finally:
            burn.kill()
            burn.wait()
        return
    runs = {}
    for tag, nproc in [("a", 1), ("b", 1)] + [(f"c{i}", 2) for i in range(reps)]:
        d = os.path.join(out, tag)
        os.makedirs(d, exist_ok=True)
        assert _run("same", d, nproc, side, "0", rt=rt) == 0, tag
        runs[tag] = torch.load(os.path.join(d, f"same_w{nproc}_r0.pt"), weights_only=True)
    diff(runs["a"], runs["b"], "w1 vs w1")
    for i in range(reps):
        diff(runs["a"], runs[f"c{i}"], f"w1 vs w2 #{i}")


if __name__ == "__main__":
    main()
