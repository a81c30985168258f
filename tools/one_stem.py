"""Run the fused ImageNet stem (forward + backward, ops/stem.py) on a synthetic
batch ``--reps`` times: the target of rocprofv3 kernel-trace / --pmc passes on
the stem kernels alone.

    python tools/one_stem.py [--batch 512] [--reps 5] [--fused 1]
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fused", type=int, default=1)
    ap.add_argument("--check", type=int, default=0,
                    help="run fwd+bwd N times from the same state, report bitwise differences")
    args = ap.parse_args()
    import zookeeper_amd.ops.stem as stem_mod
    from zookeeper_amd.nn.layers import BatchNorm, ImageStem, MaxPool2d, QuantConv2d

    stem_mod._FUSED = bool(args.fused)
    stem = ImageStem(QuantConv2d(3, 64, 7, 2, "same", kernel_initializer="he_normal"),
                     BatchNorm(64, 0.9, 1e-5, activation="relu"), MaxPool2d(3, 2, "same"),
                     BatchNorm(64, 0.9, 1e-5)).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(args.batch, 3, args.hw, args.hw, device="cuda").to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y = stem(x)
    g = torch.randn_like(y)
    y.backward(g)
    torch.cuda.synchronize()
    if args.check:
        import copy
        base = copy.deepcopy(stem.state_dict())
        ref = None
        for rep in range(args.check):
            stem.load_state_dict(base)
            for p_ in stem.parameters():
                p_.grad = None
            out = stem(x)
            out.backward(g)
            torch.cuda.synchronize()
            cur = {"out": out.detach().clone(), "running": [b.clone() for b in stem.buffers()],
                   **{n: p_.grad.clone() for n, p_ in stem.named_parameters()}}
            if ref is None:
                ref = cur
                continue
            diffs = []
            for k in cur:
                a, b = cur[k], ref[k]
                if isinstance(a, list):
                    d = max(((u.float() - v.float()).abs().max().item() for u, v in zip(a, b)),
                            default=0.0)
                else:
                    d = (a.float() - b.float()).abs().max().item()
                diffs.append(f"{k}={d:.3g}")
            print(f"rep {rep}: max |diff| vs rep 0: " + " ".join(diffs), flush=True)
    t0 = time.perf_counter()
    for _ in range(args.reps):
        y = stem(x)
        y.backward(g)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.reps * 1e3
    print(f"stem fwd+bwd b{args.batch} {args.hw}x{args.hw} fused={args.fused}: {ms:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
