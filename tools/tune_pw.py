"""Time every ``zk_igemm_dgrad`` tile variant on the 1x1 GEMMs of ResNet-50
at batch 512 (the 1x1 forward runs the dgrad kernel with its roles renamed,
the 1x1 data gradient is the kernel proper), so the default-variant
heuristic for small-K GEMMs can be set from measurements.

    python tools/tune_pw.py [--batch 512] [--reps 10] [--variants 0-17] [--dres]

Prints one line per (shape, variant): microseconds per call and the
effective HBM bandwidth of the compulsory bytes (A + output [+ dres]).
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

# (spatial size, N = output channels of the GEMM, K = reduction channels)
SHAPES = [
    (56, 64, 256), (56, 256, 64),
    (28, 128, 512), (28, 512, 128),
    (14, 256, 1024), (14, 1024, 256),
    (7, 512, 2048), (7, 2048, 512),
]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0-48")
    ap.add_argument("--dres", action="store_true", help="add a residual gradient (epilogue read)")
    args = ap.parse_args()
    lo, hi = (int(v) for v in args.variants.split("-"))
    from zookeeper_amd.ops._native import lib, stream_ptr

    L, st = lib(), stream_ptr()
    B = args.batch
    for hw, n, k in SHAPES:
        P = B * hw * hw
        a = torch.randn(P, k, device="cuda").to(torch.bfloat16)
        wt = torch.randn(1, n, k, device="cuda").to(torch.bfloat16)  # [T][N][K]
        out = torch.empty(P, n, device="cuda", dtype=torch.bfloat16)
        dres = torch.randn(P, n, device="cuda").to(torch.bfloat16) if args.dres else None
        nbytes = (a.numel() + out.numel() * (2 if args.dres else 1)) * 2
        res = []
        for v in list(range(lo, hi + 1)) + [-1]:
            def call():
                return L.zk_igemm_dgrad(a.data_ptr(), wt.data_ptr(), None,
                                        dres.data_ptr() if dres is not None else None,
                                        out.data_ptr(), B, hw, hw, n, hw, hw, k, 1, 1, 1, 0, 0,
                                        v, st)
            if call() != 0:
                continue
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            res.append((us, v))
            print(f"hw {hw:2d} N {n:4d} K {k:4d} variant {v:3d}: {us:8.1f} us "
                  f"{nbytes / us / 1e6:6.2f} TB/s", flush=True)
        best = min(r for r in res if r[1] >= 0)
        dflt = [r for r in res if r[1] == -1][0]
        print(f"== hw {hw} N {n} K {k}: best variant {best[1]} {best[0]:.1f} us, "
              f"default {dflt[0]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
