"""Standalone timings of the max-pool forward and backward (norm_pool.hip) at the
QuickNet-Large transition shapes (2x2 stride 1, valid, batch 1024) and at
ResNet's 3x3 stride 2: us per call and the HBM rate of input + output +
argmax bytes.

    python tools/pool_lab.py [--reps 20] [--tag T]
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SHAPES = [(1024, 56, 64, 2, 1, 0), (1024, 28, 128, 2, 1, 0), (1024, 14, 256, 2, 1, 0),
          (1024, 112, 64, 3, 2, 1)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from zookeeper_amd.ops._native import check, lib, stream_ptr

    L, st = lib(), stream_ptr()
    for B, H, C, k, s, p in SHAPES:
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(B, H, H, C, device="cuda").to(torch.bfloat16)
        y = torch.empty(B, Ho, Ho, C, dtype=torch.bfloat16, device="cuda")
        arg = torch.empty(B, Ho, Ho, C, dtype=torch.uint8, device="cuda")

        def run():
            check(L.zk_maxpool_fwd(x.data_ptr(), y.data_ptr(), arg.data_ptr(), B, H, H, C, Ho,
                                   Ho, k, s, p, p, 0, st), "maxpool")

        for _ in range(3):
            run()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        nbytes = x.numel() * 2 + y.numel() * 3
        print(f"{args.tag:6s} maxpool {k}x{k}/{s} B={B} {H}x{H}x{C}: {us:8.1f} us "
              f"{nbytes / us / 1e6:5.2f} TB/s", flush=True)
        dx = torch.empty_like(x)

        def run_bwd():
            check(L.zk_maxpool_bwd(y.data_ptr(), arg.data_ptr(), dx.data_ptr(), B, H, H, C, Ho,
                                   Ho, k, s, p, p, st), "maxpool_bwd")

        for _ in range(3):
            run_bwd()
        e0.record()
        for _ in range(args.reps):
            run_bwd()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.reps
        print(f"{args.tag:6s} maxpool_bwd {k}x{k}/{s} B={B} {H}x{H}x{C}: {us:8.1f} us "
              f"{nbytes / us / 1e6:5.2f} TB/s", flush=True)
        del x, y, arg, dx


if __name__ == "__main__":
    main()
