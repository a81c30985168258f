"""Time every tile variant of the binary-conv kernels on the BinaryResNet-E18
layer shapes (MI355X) and print a table; also times the library (MIOpen)
bf16 convolution backward on the same shapes for reference.

    python tools/tune_bconv.py [--batch 256] [--reps 10] [--out FILE]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from zookeeper_amd.models.binary_resnet import stage_shapes  # noqa: E402
from zookeeper_amd.nn.layers import same_padding  # noqa: E402
from zookeeper_amd.ops._native import lib, stream_ptr  # noqa: E402

DG_VARIANTS = 8
WG_VARIANTS = 8
IG_VARIANTS = list(range(18)) + list(range(20, 35)) + list(range(40, 49))
IGW_VARIANTS = list(range(13)) + list(range(20, 35))  # 20+: conv3 (3x3 s1)
IGF_VARIANTS = list(range(15)) + list(range(20, 28))
IGF4_VARIANTS = [-1] + list(range(10)) + list(range(20, 29))


def timeit(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--slab", type=int, default=1, help="wgrad split-K via workspace slabs")
    ap.add_argument("--igw", default=None, help="comma list of igemm wgrad variants (default all)")
    ap.add_argument("--tbs", default="512,1024,2048", help="wgrad target block counts")
    ap.add_argument("--only", default="fwd,dgrad,igemm,wgrad,miopen",
                    help="comma list of kernel families to time")
    args = ap.parse_args()
    fam = set(args.only.split(","))
    L, st = lib(), stream_ptr()
    B = args.batch
    shapes = sorted(set(stage_shapes((224, 224, 3))))
    results = []
    for (H, W, cin, cout, s) in shapes:
        pt, pb = same_padding(H, 3, s)
        Ho = (H + pt + pb - 3) // s + 1
        x = torch.randn(B, H, W, cin, device="cuda").to(torch.bfloat16)
        w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1, 1)
        dy = torch.randn(B, Ho, Ho, cout, device="cuda").to(torch.bfloat16)
        nwords = x.numel() // 32
        bits = torch.empty(nwords, dtype=torch.int32, device="cuda")
        mask = torch.empty_like(bits)
        sx = torch.empty_like(x)
        L.zk_sign_pack(x.data_ptr(), bits.data_ptr(), mask.data_ptr(), sx.data_ptr(), None, nwords, 1.0,
                       st)
        wbits = torch.empty(cout * 9 * cin // 32, dtype=torch.int32, device="cuda")
        wpop = torch.empty(cout * 9, dtype=torch.int32, device="cuda")
        wt = torch.empty(9, cin, cout, dtype=torch.bfloat16, device="cuda")
        L.zk_weight_pack(w.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), wt.data_ptr(), None, None, cout,
                         9, cin, st)
        dx = torch.empty_like(x)
        dw = torch.zeros(cout, 3, 3, cin, device="cuda")
        y = torch.empty(B, Ho, Ho, cout, dtype=torch.int16, device="cuda")
        stats = torch.zeros(32, 2, cout, dtype=torch.int64, device="cuda")  # striped
        flops = 2.0 * B * Ho * Ho * cout * 9 * cin
        row = {"shape": [H, W, cin, cout, s], "gflop": flops / 1e9}
        if "fwd" in fam:
            row["fwd_xnor_us"] = timeit(lambda: L.zk_bconv_fwd(
                bits.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), y.data_ptr(), stats.data_ptr(),
                B, H, W, cin, cout, 3, 3, s, pt, pt, Ho, Ho, 0, 0, st), args.reps)
        if "igf" in fam:
            wf = torch.empty(9, cout, cin, dtype=torch.bfloat16, device="cuda")
            L.zk_weight_pack(w.data_ptr(), None, None, None, wf.data_ptr(), None, cout, 9, cin, st)
            yref = None
            if "fwd" in fam:
                stats.zero_()
                L.zk_bconv_fwd(bits.data_ptr(), wbits.data_ptr(), wpop.data_ptr(), y.data_ptr(),
                               stats.data_ptr(), B, H, W, cin, cout, 3, 3, s, pt, pt, Ho, Ho, 0, 0,
                               st)
                torch.cuda.synchronize()
                yref = y.clone()
            for v in IGF_VARIANTS:
                y.zero_()
                rc = L.zk_igemm_fwd(sx.data_ptr(), wf.data_ptr(), y.data_ptr(), stats.data_ptr(),
                                    B, H, W, cin, cout, 3, 3, s, pt, pt, Ho, Ho, 0, 0, v, 32, st)
                torch.cuda.synchronize()
                if rc != 0:
                    row[f"igf_v{v}_us"] = None
                    continue
                if yref is not None:
                    row[f"igf_v{v}_exact"] = bool(torch.equal(y, yref))
                row[f"igf_v{v}_us"] = timeit(lambda: L.zk_igemm_fwd(
                    sx.data_ptr(), wf.data_ptr(), y.data_ptr(), stats.data_ptr(), B, H, W, cin,
                    cout, 3, 3, s, pt, pt, Ho, Ho, 0, 0, v, 32, st), args.reps)
        if "igf4" in fam:
            # MX-FP4 forward: e2m1 sign images, every variant checked against
            # the default one bit for bit
            sx4 = torch.empty(B, H, W, cin // 2, dtype=torch.uint8, device="cuda")
            L.zk_sign_pack(x.data_ptr(), None, None, None, sx4.data_ptr(), nwords, 1.0, st)
            wf4 = torch.empty(9, cout, cin // 2, dtype=torch.uint8, device="cuda")
            L.zk_weight_pack(w.data_ptr(), None, None, None, None, wf4.data_ptr(), cout, 9, cin,
                             st)
            yref4 = None
            for v in IGF4_VARIANTS:
                y.zero_()
                rc = L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(),
                                        stats.data_ptr(), B, H, W, cin, cout, 3, 3, s, pt, pt, Ho,
                                        Ho, 0, 0, v, 32, st)
                torch.cuda.synchronize()
                if rc != 0:
                    row[f"igf4_v{v}_us"] = None
                    continue
                if yref4 is None:
                    yref4 = y.clone()
                else:
                    row[f"igf4_v{v}_exact"] = bool(torch.equal(y, yref4))
                row[f"igf4_v{v}_us"] = timeit(lambda: L.zk_igemm_fwd_fp4(
                    sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(), stats.data_ptr(), B, H, W, cin,
                    cout, 3, 3, s, pt, pt, Ho, Ho, 0, 0, v, 32, st), args.reps)
        ref_dx = None
        for v in (range(DG_VARIANTS) if ("dgrad" in fam or "igemm" in fam) else ()):
            if "dgrad" not in fam and v != 7:
                continue
            rc = L.zk_bconv_dgrad(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(), None,
                                  dx.data_ptr(), B, H, W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, v, st)
            if rc != 0:
                row[f"dgrad_v{v}_us"] = None
                torch.cuda.synchronize()
                continue
            row[f"dgrad_v{v}_us"] = timeit(lambda: L.zk_bconv_dgrad(
                dy.data_ptr(), wt.data_ptr(), mask.data_ptr(), None, dx.data_ptr(), B, H, W, cin,
                Ho, Ho, cout, 3, 3, s, pt, pt, v, st), args.reps)
            if v == 7:
                torch.cuda.synchronize()
                ref_dx = dx.float().clone()
        for v in (IG_VARIANTS if "igemm" in fam else ()):
            dx.zero_()
            rc = L.zk_igemm_dgrad(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(), None,
                                  dx.data_ptr(), B, H, W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, v, st)
            torch.cuda.synchronize()
            if rc != 0:
                row[f"igd_v{v}_us"] = None
                continue
            if ref_dx is not None:
                row[f"igd_v{v}_maxerr"] = (dx.float() - ref_dx).abs().max().item()
            row[f"igd_v{v}_us"] = timeit(lambda: L.zk_igemm_dgrad(
                dy.data_ptr(), wt.data_ptr(), mask.data_ptr(), None, dx.data_ptr(), B, H, W, cin,
                Ho, Ho, cout, 3, 3, s, pt, pt, v, st), args.reps)
        ref_dw = None
        for v in (range(WG_VARIANTS) if ("wgrad" in fam or "igw" in fam) else ()):
            if "wgrad" not in fam and v != 5:
                continue
            for tb in (512, 1024, 2048):
                rc = L.zk_bconv_wgrad(dy.data_ptr(), bits.data_ptr(), w.data_ptr(), dw.data_ptr(),
                                      B, H, W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, 0, 1.0, tb, v, st)
                if rc != 0:
                    row[f"wgrad_v{v}_tb{tb}_us"] = None
                    continue
                row[f"wgrad_v{v}_tb{tb}_us"] = timeit(lambda: L.zk_bconv_wgrad(
                    dy.data_ptr(), bits.data_ptr(), w.data_ptr(), dw.data_ptr(), B, H, W, cin, Ho,
                    Ho, cout, 3, 3, s, pt, pt, 0, 1.0, tb, v, st), args.reps)
                if ref_dw is None:
                    dw.zero_()
                    L.zk_bconv_wgrad(dy.data_ptr(), bits.data_ptr(), w.data_ptr(), dw.data_ptr(),
                                     B, H, W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, 0, 1.0, tb, v, st)
                    torch.cuda.synchronize()
                    ref_dw = dw.clone()
        igw = [int(v) for v in args.igw.split(",")] if args.igw else IGW_VARIANTS
        for v in (igw if "igw" in fam else ()):
            fn = L.zk_igemm_wgrad
            sxp = sx.data_ptr()
            for tb in [int(t) for t in args.tbs.split(",")]:
                dw.zero_()
                nb = L.zk_igemm_wgrad_ws_bytes(B, cin, H, W, Ho, Ho, cout, 3, 3, s, pt, pt, tb, v)
                wsb = torch.empty(max(nb, 4) // 4, device="cuda") if args.slab else None
                wsp = wsb.data_ptr() if wsb is not None else None
                wsn = wsb.numel() * 4 if wsb is not None else 0
                rc = fn(dy.data_ptr(), sxp, w.data_ptr(), dw.data_ptr(),
                        B, H, W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, 0, 1.0, tb, v, wsp, wsn, st)
                torch.cuda.synchronize()
                if rc != 0:
                    row[f"igw_v{v}_tb{tb}_us"] = None
                    continue
                if ref_dw is None:
                    ref_dw = dw.clone()  # first variant that ran: the reference
                else:
                    row[f"igw_v{v}_tb{tb}_relerr"] = ((dw - ref_dw).abs().max() /
                                                      ref_dw.abs().max()).item()
                row[f"igw_v{v}_tb{tb}_us"] = timeit(lambda: fn(
                    dy.data_ptr(), sxp, w.data_ptr(), dw.data_ptr(), B, H, W, cin, Ho,
                    Ho, cout, 3, 3, s, pt, pt, 0, 1.0, tb, v, wsp, wsn, st), args.reps)
        # library reference: bf16 conv backward on unpacked ±1 operands
        xs = torch.where(x >= 0, 1.0, -1.0).to(torch.bfloat16).permute(0, 3, 1, 2)
        wsn = torch.where(w >= 0, 1.0, -1.0).to(torch.bfloat16).permute(0, 3, 1, 2)
        if s == 1 and "miopen" in fam:
            row["miopen_bwd_us"] = timeit(lambda: torch.ops.aten.convolution_backward(
                dy.permute(0, 3, 1, 2), xs, wsn, None, (1, 1), (1, 1), (1, 1), False, (0, 0), 1,
                (True, True, False)), args.reps)
        dgs = [row[k] for k in row if (k.startswith("dgrad_v") or k.startswith("igd_v"))
               and k.endswith("_us") and row[k]]
        wgs = [row[k] for k in row if (k.startswith("wgrad_v") or k.startswith("igw_v"))
               and k.endswith("_us") and row[k]]
        if dgs:
            row["best_dgrad_tflops"] = flops / min(dgs) / 1e6
        if wgs:
            row["best_wgrad_tflops"] = flops / min(wgs) / 1e6
        results.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
