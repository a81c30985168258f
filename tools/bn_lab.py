"""Standalone timings of the streaming BatchNorm kernels (batchnorm.hip,
norm_pool.hip) at the E18 (batch 1536) and ResNet-50 (batch 1024) shapes:
per-call us and the effective HBM rate of the bytes each call must move.

    python tools/bn_lab.py [--reps 20] [--json gpurun_out/bn_lab.jsonl]
"""

import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

E18 = [(1536 * 56 * 56, 64), (1536 * 28 * 28, 128), (1536 * 14 * 14, 256), (1536 * 7 * 7, 512)]
R50 = [(1024 * 56 * 56, 64), (1024 * 56 * 56, 256), (1024 * 28 * 28, 128),
       (1024 * 28 * 28, 512), (1024 * 14 * 14, 256), (1024 * 14 * 14, 1024),
       (1024 * 7 * 7, 512), (1024 * 7 * 7, 2048)]


def timed(fn, reps):
    for _ in range(3):
        fn()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default="")
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    from zookeeper_amd.ops._native import check, lib, stream_ptr

    L, st = lib(), stream_ptr()
    dev = "cuda"
    rows = []

    def report(kernel, P, C, us, nbytes):
        r = {"tag": args.tag, "kernel": kernel, "P": P, "C": C, "us": round(us, 1),
             "TBps": round(nbytes / us / 1e6, 2)}
        rows.append(r)
        print(f"{kernel:28s} P={P:>9d} C={C:>5d} {us:8.1f} us {r['TBps']:5.2f} TB/s", flush=True)

    # ceilings: a device copy (read n + write n bytes) and a read-only sum,
    # 1.6 GB per tensor
    src = torch.randn(1024 * 56 * 56, 256, device=dev).to(torch.bfloat16)
    dst = torch.empty_like(src)
    n = src.numel()
    report("ceiling: torch copy_", src.shape[0], 256, timed(lambda: dst.copy_(src), args.reps),
           4 * n)
    report("ceiling: torch sum (read)", src.shape[0], 256,
           timed(lambda: src.sum(dtype=torch.float32), args.reps), 2 * n)
    del src, dst
    for P, C in E18:
        g = torch.randn(P, C, device=dev).to(torch.bfloat16)
        y = torch.randint(-300, 300, (P, C), dtype=torch.int16, device=dev)
        res = torch.randn(P, C, device=dev).to(torch.bfloat16)
        out = torch.empty_like(res)
        dy = torch.empty_like(res)
        coef = torch.rand(3 * C, device=dev)
        sc = torch.rand(C, device=dev)
        sh = torch.rand(C, device=dev)
        mask = torch.empty(P * C // 8, dtype=torch.uint8, device=dev)
        sx4 = torch.empty(P, C // 2, dtype=torch.uint8, device=dev)
        n = P * C
        us = timed(lambda: check(L.zk_bn_bwd_dx(g.data_ptr(), y.data_ptr(), coef.data_ptr(),
                                                dy.data_ptr(), P, C, 0, st), "dx"), args.reps)
        report("bn_bwd_dx (int16 y)", P, C, us, 6 * n)
        us = timed(lambda: check(L.zk_bn_apply_sign(
            y.data_ptr(), sc.data_ptr(), sh.data_ptr(), res.data_ptr(), out.data_ptr(), None,
            mask.data_ptr(), sx4.data_ptr(), 1.0, P, C, st), "apply"), args.reps)
        report("bn_apply_sign (+res, sx4)", P, C, us, n * (2 + 2 + 2 + 0.5 + 0.125))
        mean = torch.rand(C, device=dev)
        rstd = torch.rand(C, device=dev)
        sums = torch.zeros(2 * C * 512, device=dev)
        us = timed(lambda: check(L.zk_bn_bwd_reduce(g.data_ptr(), y.data_ptr(), mean.data_ptr(),
                                                    rstd.data_ptr(), sums.data_ptr(), P, C, 512,
                                                    st), "reduce"), args.reps)
        report("bn_bwd_reduce (int16 y)", P, C, us, 4 * n)
        hw = {64: 56, 128: 28, 256: 14, 512: 7}[C]
        if hw % 2 == 0:
            pooled = torch.empty(P // 4, C, dtype=torch.bfloat16, device=dev)
            us = timed(lambda: check(L.zk_bn_apply_sign_pool(
                y.data_ptr(), sc.data_ptr(), sh.data_ptr(), res.data_ptr(), out.data_ptr(), None,
                mask.data_ptr(), sx4.data_ptr(), 1.0, pooled.data_ptr(), P // (hw * hw), hw, hw,
                C, st), "apply_pool"), args.reps)
            report("bn_apply_sign_pool", P, C, us, n * (2 + 2 + 2 + 0.5 + 0.125 + 0.5))
            del pooled
        del g, y, res, out, dy, mask, sx4
    for P, C in R50:
        g = torch.randn(P, C, device=dev).to(torch.bfloat16)
        x = torch.randn(P, C, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(x)
        m = torch.randint(0, 255, (P * C // 8,), dtype=torch.uint8, device=dev)
        bcoef = torch.rand(3 * C, device=dev)
        fcoef = torch.rand(4 * C, device=dev)
        n = P * C
        us = timed(lambda: check(L.zk_bn_bwd_dx_bf16(g.data_ptr(), x.data_ptr(), m.data_ptr(),
                                                     bcoef.data_ptr(), dx.data_ptr(), P, C, st),
                                 "dxbf"), args.reps)
        report("bn_bwd_dx_bf16 (mask)", P, C, us, n * (6 + 0.125))
        us = timed(lambda: check(L.zk_bn_bwd_dx_relu_bf16(
            g.data_ptr(), x.data_ptr(), fcoef.data_ptr(), bcoef.data_ptr(), dx.data_ptr(), P, C,
            st), "dxrelu"), args.reps)
        report("bn_bwd_dx_relu_bf16", P, C, us, n * 6)
        parts = torch.zeros(2 * C * 512, device=dev)
        npart = ctypes.c_int(0)
        us = timed(lambda: check(L.zk_bn_bwd_reduce_bf16_parts(
            g.data_ptr(), x.data_ptr(), m.data_ptr(), fcoef.data_ptr(), parts.data_ptr(), P, C,
            ctypes.byref(npart), st), "reduce_bf16"), args.reps)
        report("bn_bwd_reduce_bf16_parts", P, C, us, n * (4 + 0.125))
        us = timed(lambda: check(L.zk_bn_apply_bf16(x.data_ptr(), fcoef.data_ptr(),
                                                    dx.data_ptr(), P, C, 1, st), "apbf"),
                   args.reps)
        report("bn_apply_bf16 (relu)", P, C, us, n * 4)
        tiles = (P + 255) // 256  # a 256-row GEMM tile's epilogue rows
        rows_t = torch.zeros(tiles, 2 * C, device=dev)
        us = timed(lambda: check(L.zk_bn_bwd_tiles_reduce(rows_t.data_ptr(), tiles, C,
                                                          parts.data_ptr(), st), "tiles"),
                   args.reps)
        report("bn_bwd_tiles_reduce", tiles, C, us, tiles * 2 * C * 8 + 2 * C * 512 * 4)
        del g, x, dx, m, rows_t
    if args.json:
        os.makedirs(os.path.dirname(args.json) or ".", exist_ok=True)
        with open(args.json, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
