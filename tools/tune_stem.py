"""Time the fused-stem kernels (stem.hip) at BinaryResNet-E18 shapes
(batch 256, 224x224x3 -> 112x112x64 -> 56x56x64) and the library path.

    python tools/tune_stem.py [--batch 256] [--reps 10]
"""

import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from zookeeper_amd.ops._native import lib, stream_ptr  # noqa: E402


def timeit(fn, reps):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    L, st = lib(), stream_ptr()
    B, H, W, Cin, Cout, K, s = args.batch, 224, 224, 3, 64, 7, 2
    pt, pl, Ho, Wo = 2, 2, 112, 112
    Hp, Wp = (Ho - 1) * s + K, (Wo - 1) * s + 8
    Wp += Wp % 2
    x = torch.randn(B, H, W, Cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(Cout, K, K, Cin, device="cuda") * 0.1
    xp = torch.empty(B, Hp, Wp, 4, dtype=torch.bfloat16, device="cuda")
    ws = torch.empty(K, Cout, 32, dtype=torch.bfloat16, device="cuda")
    y1 = torch.empty(B, Ho, Wo, Cout, dtype=torch.bfloat16, device="cuda")
    part = torch.empty(L.zk_stem_max_parts(B, Ho, Wo), 2, Cout, device="cuda")
    nb = ctypes.c_int(0)
    row = {}
    row["pack_input_us"] = timeit(lambda: L.zk_stem_pack_input(
        x.data_ptr(), xp.data_ptr(), B, H, W, Cin, Hp, Wp, pt, pl, st), args.reps)
    L.zk_stem_pack_weight(w.data_ptr(), ws.data_ptr(), Cout, K, K, Cin, st)
    for v in range(4):
        y1.fill_(0)
        L.zk_stem_conv_fwd(xp.data_ptr(), ws.data_ptr(), y1.data_ptr(), part.data_ptr(), B, Cin,
                           Cout, K, K, s, Ho, Wo, Hp, Wp, v, ctypes.byref(nb), st)
        torch.cuda.synchronize()
        row[f"conv_fwd_v{v}_us"] = timeit(lambda: L.zk_stem_conv_fwd(
            xp.data_ptr(), ws.data_ptr(), y1.data_ptr(), part.data_ptr(), B, Cin, Cout, K, K, s,
            Ho, Wo, Hp, Wp, v, ctypes.byref(nb), st), args.reps)
        print(f"conv_fwd v{v}: {row[f'conv_fwd_v{v}_us']:.1f} us", flush=True)
    coef = torch.empty(4, Cout, device="cuda")
    rm, rv = torch.zeros(Cout, device="cuda"), torch.ones(Cout, device="cuda")
    L.zk_stem_conv_fwd(xp.data_ptr(), ws.data_ptr(), y1.data_ptr(), part.data_ptr(), B, Cin, Cout,
                       K, K, s, Ho, Wo, Hp, Wp, 0, ctypes.byref(nb), st)
    row["finalize_us"] = timeit(lambda: L.zk_bn_finalize_partials(
        part.data_ptr(), nb.value, Cout, float(B * Ho * Wo), None, None, 1e-5, 0.9,
        rm.data_ptr(), rv.data_ptr(), coef.data_ptr(), st), args.reps)
    fws = torch.empty(L.zk_bn_finalize_ws_bytes(Cout) // 8, dtype=torch.float64, device="cuda")
    coef2 = torch.empty_like(coef)
    row["finalize_ws_us"] = timeit(lambda: L.zk_bn_finalize_partials_ws(
        part.data_ptr(), nb.value, Cout, float(B * Ho * Wo), None, None, 1e-5, 0.9,
        rm.data_ptr(), rv.data_ptr(), coef2.data_ptr(), fws.data_ptr(), st), args.reps)
    row["finalize_ws_coef_maxrel"] = ((coef2 - coef).abs() / coef.abs().clamp_min(1e-12)).max().item()
    print(f"finalize {row['finalize_us']:.1f} us, two-pass {row['finalize_ws_us']:.1f} us",
          flush=True)
    H2, W2 = 56, 56
    p = torch.empty(B, H2, W2, Cout, dtype=torch.bfloat16, device="cuda")
    arg = torch.empty(B, H2, W2, Cout, dtype=torch.uint8, device="cuda")
    part2 = torch.empty(L.zk_stem_max_pool_parts(), 2, Cout, device="cuda")
    nb2 = ctypes.c_int(0)
    row["pool_fwd_us"] = timeit(lambda: L.zk_stem_pool_fwd(
        y1.data_ptr(), coef.data_ptr(), p.data_ptr(), arg.data_ptr(), part2.data_ptr(), B, Ho, Wo,
        Cout, H2, W2, 3, 2, 0, 0, ctypes.byref(nb2), st), args.reps)
    dp = torch.randn(B, H2, W2, Cout, device="cuda").to(torch.bfloat16)
    row["pool_bwd_sums_us"] = timeit(lambda: L.zk_stem_pool_bwd_sums(
        dp.data_ptr(), arg.data_ptr(), y1.data_ptr(), p.data_ptr(), coef.data_ptr(),
        part2.data_ptr(), B, Ho,
        Wo, Cout, H2, W2, 3, 2, 0, 0, ctypes.byref(nb2), st), args.reps)
    bcoef = torch.randn(3, Cout, device="cuda")
    dy1 = torch.empty_like(y1)
    row["dy1_us"] = timeit(lambda: L.zk_stem_dy1(
        dp.data_ptr(), arg.data_ptr(), y1.data_ptr(), coef.data_ptr(), bcoef.data_ptr(),
        dy1.data_ptr(), B, Ho, Wo, Cout, H2, W2, 3, 2, 0, 0, st), args.reps)
    dw = torch.zeros(Cout, K, K, Cin, device="cuda")
    for tb in (256, 512, 1024, 2048):
        row[f"wgrad_tb{tb}_us"] = timeit(lambda: L.zk_stem_wgrad(
            dy1.data_ptr(), xp.data_ptr(), dw.data_ptr(), None, B, Cin, Cout, K, K, s, Ho, Wo, Hp, Wp,
            tb, st), args.reps)
    # library reference: conv fwd + wgrad on the same shapes
    xn = x.permute(0, 3, 1, 2)
    wn = w.permute(0, 3, 1, 2).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xpad = torch.nn.functional.pad(xn, (2, 3, 2, 3)).contiguous(memory_format=torch.channels_last)
    row["miopen_fwd_us"] = timeit(lambda: torch.nn.functional.conv2d(xpad, wn, stride=2),
                                  args.reps)
    gy = dy1.permute(0, 3, 1, 2)
    row["miopen_wgrad_us"] = timeit(lambda: torch.ops.aten.convolution_backward(
        gy, xpad, wn, None, (2, 2), (0, 0), (1, 1), False, (0, 0), 1, (False, True, False)),
        args.reps)
    print(json.dumps(row, indent=1))


if __name__ == "__main__":
    main()
