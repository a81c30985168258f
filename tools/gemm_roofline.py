"""Binary-conv GEMMs of BinaryResNet-E18 against their rooflines (MI355X).

For every distinct layer shape at ``--batch`` (default 1024, the bench
default), time the default kernel of each pass -- MX-FP4 forward, data
gradient (with STE mask + residual gradient, as in the step), weight
gradient (slab split-K + reduce) -- and print

* us per call, PF/s of the GEMM (2*M*N*K),
* the compute floor (bf16 MFMA 2.5 PF dense; fp4 forward 10 PF) and the HBM
  floor (the bytes the pass must move at 6.0 TB/s achievable),
* ``x floor`` = time / max(compute floor, HBM floor).

    python tools/gemm_roofline.py [--batch 1024] [--reps 10] [--json out.json]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

BF16_PEAK = 2.5e15
FP4_PEAK = 10e15
HBM = 6.0e12


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
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    ap.add_argument("--ops", default="fwd4,dgrad,wgrad")
    ap.add_argument("--dvariant", type=int, default=-1)
    ap.add_argument("--wvariant", type=int, default=-1)
    ap.add_argument("--shapes", default="all", help="all or H+W+Cin+Cout+s/... ('+' or ',')")
    ap.add_argument("--dvariants", default=None, help="dgrad variants to compare (+-separated)")
    ap.add_argument("--wvariants", default=None, help="wgrad variants to compare (+-separated)")
    ap.add_argument("--wgrad-mode", default="atomic", choices=["atomic", "slab"],
                    help="split-K reduction: fp32 atomics into dW (default mode) or slabs + "
                         "the fixed-order reduce (deterministic mode)")
    args = ap.parse_args()
    from zookeeper_amd.models.binary_resnet import stage_shapes
    from zookeeper_amd.nn.layers import same_padding
    from zookeeper_amd.ops._native import lib, stream_ptr

    L, st = lib(), stream_ptr()
    B = args.batch
    slab = args.wgrad_mode == "slab"
    if args.shapes == "all":
        shapes = sorted(set(stage_shapes((224, 224, 3))), key=lambda s: (-s[0], s[2], s[4]))
    else:
        shapes = [tuple(int(v) for v in s.replace("+", ",").split(","))
                  for s in args.shapes.split("/")]
    rows = []
    tot = {"fwd4": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    counts = {}
    for shp in stage_shapes((224, 224, 3)):
        counts[shp] = counts.get(shp, 0) + 1
    for (H, W, cin, cout, s) in shapes:
        pt, pb = same_padding(H, 3, s)
        Ho = (H + pt + pb - 3) // s + 1
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(B, H, W, cin, device="cuda", generator=g).to(torch.bfloat16)
        w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1, 1, generator=g)
        dy = torch.randn(B, Ho, Ho, cout, device="cuda", generator=g).to(torch.bfloat16)
        nwords = x.numel() // 32
        mask = torch.empty(nwords, dtype=torch.int32, device="cuda")
        sx = torch.empty_like(x)
        sx4 = torch.empty(B, H, W, cin // 2, dtype=torch.uint8, device="cuda")
        L.zk_sign_pack(x.data_ptr(), None, mask.data_ptr(), sx.data_ptr(), sx4.data_ptr(), nwords,
                       1.0, st)
        wt = torch.empty(9, cin, cout, dtype=torch.bfloat16, device="cuda")
        wf4 = torch.empty(9, cout, cin // 2, dtype=torch.uint8, device="cuda")
        L.zk_weight_pack(w.data_ptr(), None, None, wt.data_ptr(), None, wf4.data_ptr(), cout, 9,
                         cin, st)
        dx = torch.empty_like(x)
        dres = torch.randn(x.shape, device="cuda", generator=g).to(torch.bfloat16)
        dw = torch.zeros(cout, 3, 3, cin, device="cuda")
        y = torch.empty(B, Ho, Ho, cout, dtype=torch.int16, device="cuda")
        stats = torch.zeros(32, 2, cout, dtype=torch.int64, device="cuda")
        nb = L.zk_igemm_wgrad_ws_bytes(B, cin, H, W, Ho, Ho, cout, 3, 3, s, pt, pt, 0,
                                       args.wvariant)
        ws = torch.empty(max(nb, 4) // 4, device="cuda")
        flops = 2.0 * B * Ho * Ho * cout * 9 * cin
        S_in = B * H * W * cin * 2  # bf16 bytes of an input-sized activation
        S_out = B * Ho * Ho * cout * 2

        def fwd4():
            assert L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(),
                                      stats.data_ptr(), B, H, W, cin, cout, 3, 3, s, pt, pt, Ho,
                                      Ho, 0, 0, -1, 32, st) == 0

        def dgrad():
            assert L.zk_igemm_dgrad(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(),
                                    dres.data_ptr(), dx.data_ptr(), B, H, W, cin, Ho, Ho, cout, 3,
                                    3, s, pt, pt, args.dvariant, st) == 0

        def wgrad():
            assert L.zk_igemm_wgrad(dy.data_ptr(), sx.data_ptr(), w.data_ptr(), dw.data_ptr(), B,
                                    H, W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, 0, 1.0, 0,
                                    args.wvariant, ws.data_ptr() if slab else None,
                                    ws.numel() * 4 if slab else 0, st) == 0

        # bytes each pass must move through HBM at least
        need = {"fwd4": (S_in / 4 + S_out, FP4_PEAK),        # sx4 in, int16 y out
                "dgrad": (S_out + 2 * S_in + S_in / 16, BF16_PEAK),  # dy, dres, dx, mask
                "wgrad": (S_out + S_in, BF16_PEAK)}          # dy, sx
        fns = {"fwd4": fwd4, "dgrad": dgrad, "wgrad": wgrad}
        runs = []
        for op in args.ops.split(","):
            vs = {"dgrad": args.dvariants, "wgrad": args.wvariants}.get(op)
            for v in ([int(x) for x in vs.split("+")] if vs else [None]):
                runs.append((op, v))
        for op, v in runs:
            if v is not None:
                if op == "dgrad":
                    args.dvariant = v
                else:
                    args.wvariant = v
                    nb = L.zk_igemm_wgrad_ws_bytes(B, cin, H, W, Ho, Ho, cout, 3, 3, s, pt, pt, 0, v)
                    ws = torch.empty(max(nb, 4) // 4, device="cuda")
            try:
                us = timeit(fns[op], args.reps)
            except AssertionError:
                print(f"{op} v{v}: unsupported for this shape", flush=True)
                continue
            nbytes, peak = need[op]
            t_c, t_m = flops / peak * 1e6, nbytes / HBM * 1e6
            rec = {"op": op, "variant": v, "shape": [H, W, cin, cout, s], "us": round(us, 1),
                   "pflops": round(flops / us / 1e9, 3), "gbps": round(nbytes / us / 1e3, 1),
                   "floor_compute_us": round(t_c, 1), "floor_hbm_us": round(t_m, 1),
                   "x_floor": round(us / max(t_c, t_m), 2), "layers": counts.get((H, W, cin, cout, s), 0)}
            rows.append(rec)
            if v is None:
                tot[op] += us * rec["layers"]
            print(f"{op:6s}{'' if v is None else ' v' + str(v):5s} {H:3d}x{W:<3d} {cin:4d}->{cout:<4d} s{s}  {us:8.1f} us  "
                  f"{rec['pflops']:6.3f} PF/s  {rec['gbps']:7.1f} GB/s  floor c {t_c:6.1f} "
                  f"m {t_m:6.1f}  x{rec['x_floor']:.2f}  (x{rec['layers']} layers)", flush=True)
        del x, dy, dx, dres, sx, sx4, ws, y
        torch.cuda.empty_cache()
    print("per-step totals (us, all 16 binary convs): " +
          ", ".join(f"{k} {v:.0f}" for k, v in tot.items() if v), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"batch": B, "rows": rows, "totals_us": tot}, f, indent=1)


if __name__ == "__main__":
    main()
