"""Time every ``zk_igemm_fwd_bf16`` tile variant on the float 3x3 convolutions
of ResNet-50 (bottleneck conv2, stride 1 and the stride-2 stage entries) at
one batch, next to the default (-1), so the default-variant rule can be set
from measurements.

    python tools/tune_fwd_bf16.py [--batch 1024] [--reps 10] [--variants 0-5]
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

# (input spatial size, channels, stride): ResNet-50 conv2 of each stage
SHAPES = [(56, 64, 1), (56, 128, 2), (28, 128, 1), (28, 256, 2), (14, 256, 1), (14, 512, 2),
          (7, 512, 1)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--variants", default="0-5")
    args = ap.parse_args()
    lo, hi = (int(v) for v in args.variants.split("-"))
    from zookeeper_amd.nn.layers import same_padding
    from zookeeper_amd.ops._native import lib, stream_ptr

    L, st = lib(), stream_ptr()
    B = args.batch
    for hw, c, s in SHAPES:
        pt, pb = same_padding(hw, 3, s)
        ho = (hw + pt + pb - 3) // s + 1
        x = torch.randn(B, hw, hw, c, device="cuda").to(torch.bfloat16)
        wf = (torch.randn(9, c, c, device="cuda") * 0.05).to(torch.bfloat16)
        y = torch.empty(B, ho, ho, c, dtype=torch.bfloat16, device="cuda")
        res = []
        for v in list(range(lo, hi + 1)) + [-1]:
            if not L.zk_igemm_fwd_bf16_supported(B, hw, hw, c, c, 3, 3, s, pt, pt, ho, ho, v):
                continue

            def run():
                rc = L.zk_igemm_fwd_bf16(x.data_ptr(), wf.data_ptr(), y.data_ptr(), B, hw, hw,
                                         c, c, 3, 3, s, pt, pt, ho, ho, 0, v, st)
                assert rc == 0, rc

            for _ in range(2):
                run()
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.reps
            flops = 2.0 * B * ho * ho * c * 9 * c
            print(f"hw {hw:3d} C {c:4d} s {s} variant {v:3d}: {us:8.1f} us "
                  f"{flops / us / 1e9:6.2f} PFLOP/s", flush=True)
            res.append((us, v))
        best = min(r for r in res if r[1] >= 0)
        dflt = [r for r in res if r[1] == -1]
        print(f"== hw {hw} C {c} s {s}: best variant {best[1]} {best[0]:.1f} us, "
              f"default {dflt[0][0] if dflt else float('nan'):.1f} us", flush=True)
        del x, wf, y


if __name__ == "__main__":
    main()
