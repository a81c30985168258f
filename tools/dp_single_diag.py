"""Diagnose the forced-DP (1-rank RCCL) vs plain-run difference of
tests/gpu/test_dp_gpu.py: run tests/dp_gpu_worker.py in several
configurations and print each one's relative parameter error against the
plain run of the same options.

    python -m tools.dp_single_diag [side=0] [reps=2]
"""
import os
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dp_gpu_worker.py")


def run(out, side, force, rt="", extra=None, steps="2"):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4", ZK_TEST_SIDE=side,
               ZK_TEST_STEPS=steps,
               ZK_TEST_GRAPH="0", ZK_TEST_FORCE_DP="1" if force else "0",
               ZK_TEST_BACKEND="nccl" if force else "gloo", ZK_TEST_RT=rt)
    env.update(extra or {})
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    rc = subprocess.run([sys.executable, WORKER, "same", out], env=env, timeout=240).returncode
    assert rc == 0, rc
    return torch.load(os.path.join(out, "same_w1dp_r0.pt" if force else "same_w1_r0.pt"),
                      weights_only=True)


def main():
    args = dict(a.split("=") for a in sys.argv[1:])
    side, reps = args.get("side", "0"), int(args.get("reps", "2"))
    steps = args.get("steps", "2")
    cfgs = [("", None), ("", {"ZK_COMM_HOST_SYNC": "1"}), ("dgrad_rw=0", None),
            ("deterministic=1", None)]
    if "only" in args:
        cfgs = [cfgs[int(i)] for i in args["only"].split("+")]
    for rt, extra in cfgs:
        for r in range(reps):
            with tempfile.TemporaryDirectory() as d:
                ref = run(d, side, False, rt, steps=steps)
                if args.get("refref") == "1":
                    # plain vs plain: the run-to-run noise floor
                    os.rename(os.path.join(d, "same_w1_r0.pt"), os.path.join(d, "ref0.pt"))
                    dp = run(d, side, False, rt, extra, steps=steps)
                else:
                    dp = run(d, side, True, rt, extra, steps=steps)
            upd = (ref["params"] - ref["init"]).norm().item()
            err = (dp["params"] - ref["params"]).norm().item() / upd
            diff = (dp["params"] - ref["params"]).abs()
            worst = []
            step_ref = ref["params"] - ref["init"]
            for name, off, n in ref["slots"]:
                m = diff[off:off + n].norm().item()
                rel = m / max(step_ref[off:off + n].norm().item(), 1e-30)
                if rel > 1e-4:
                    worst.append((rel, name))
            worst.sort(reverse=True)
            print(f"side={side} steps={steps} rt={rt or '-'} extra={extra} rep={r}: err={err:.3g} "
                  f"n_bad={len(worst)} worst_rel={[(f'{m:.2e}', n) for m, n in worst[:10]]}",
                  flush=True)


if __name__ == "__main__":
    main()
