"""Run one binary-conv kernel (default variant unless --variant) on one E18
layer shape, ``--reps`` times back to back: the target of rocprofv3 --pmc
passes on a single kernel.

    python tools/one_conv.py --op dgrad --shape 56,56,64,64,1 [--variant -1] [--reps 20]
    rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... -- python tools/one_conv.py --op dgrad ...
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--op", choices=["dgrad", "wgrad", "fwd4"], default="dgrad")
    ap.add_argument("--shape", default="56,56,64,64,1", help="H,W,Cin,Cout,stride")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-y", action="store_true",
                    help="fwd4: statistics only, no int16 y stores (lab option 9)")
    args = ap.parse_args()
    from zookeeper_amd.nn.layers import same_padding
    from zookeeper_amd.ops._native import lib, stream_ptr

    if args.shape == "all":
        from zookeeper_amd.models.binary_resnet import stage_shapes

        for shp in sorted(set(stage_shapes((224, 224, 3)))):
            run_one(args, ",".join(str(v) for v in shp))
        return
    run_one(args, args.shape)


def run_one(args, shape: str) -> None:
    from zookeeper_amd.nn.layers import same_padding
    from zookeeper_amd.ops._native import lib, stream_ptr

    H, W, cin, cout, s = (int(v) for v in shape.replace("x", ",").split(","))
    B = args.batch
    L, st = lib(), stream_ptr()
    pt, pb = same_padding(H, 3, s)
    Ho = (H + pt + pb - 3) // s + 1
    x = torch.randn(B, H, W, cin, device="cuda").to(torch.bfloat16)
    w = torch.empty(cout, 3, 3, cin, device="cuda").uniform_(-1, 1)
    dy = torch.randn(B, Ho, Ho, cout, device="cuda").to(torch.bfloat16)
    nwords = x.numel() // 32
    mask = torch.empty(nwords, dtype=torch.int32, device="cuda")
    sx = torch.empty_like(x)
    sx4 = torch.empty(B, H, W, cin // 2, dtype=torch.uint8, device="cuda")
    L.zk_sign_pack(x.data_ptr(), None, mask.data_ptr(), sx.data_ptr(), sx4.data_ptr(), nwords,
                   1.0, st)
    wt = torch.empty(9, cin, cout, dtype=torch.bfloat16, device="cuda")
    wf = torch.empty(9, cout, cin, dtype=torch.bfloat16, device="cuda")
    wf4 = torch.empty(9, cout, cin // 2, dtype=torch.uint8, device="cuda")
    L.zk_weight_pack(w.data_ptr(), None, None, wt.data_ptr(), wf.data_ptr(), wf4.data_ptr(), cout,
                     9, cin, st)
    dx = torch.empty_like(x)
    dres = torch.randn_like(x)
    dw = torch.zeros(cout, 3, 3, cin, device="cuda")
    y = torch.empty(B, Ho, Ho, cout, dtype=torch.int16, device="cuda")
    stats = torch.zeros(32, 2, cout, dtype=torch.int64, device="cuda")
    nb = L.zk_igemm_wgrad_ws_bytes(B, cin, H, W, Ho, Ho, cout, 3, 3, s, pt, pt, 0, args.variant)
    ws = torch.empty(max(nb, 4) // 4, device="cuda")

    def run():
        if args.op == "dgrad":
            rc = L.zk_igemm_dgrad(dy.data_ptr(), wt.data_ptr(), mask.data_ptr(), dres.data_ptr(),
                                  dx.data_ptr(), B, H, W, cin, Ho, Ho, cout, 3, 3, s, pt, pt,
                                  args.variant, st)
        elif args.op == "wgrad":
            rc = L.zk_igemm_wgrad(dy.data_ptr(), sx.data_ptr(), w.data_ptr(), dw.data_ptr(), B, H,
                                  W, cin, Ho, Ho, cout, 3, 3, s, pt, pt, 0, 1.0, 0, args.variant,
                                  ws.data_ptr(), ws.numel() * 4, st)
        else:
            rc = L.zk_igemm_fwd_fp4(sx4.data_ptr(), wf4.data_ptr(), y.data_ptr(), stats.data_ptr(),
                                    B, H, W, cin, cout, 3, 3, s, pt, pt, Ho, Ho, 0, 0,
                                    args.variant, 32, st)
        assert rc == 0, rc

    L.zk_set_option(9, int(args.no_y))
    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        run()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / args.reps * 1e6
    flops = 2.0 * B * Ho * Ho * cout * 9 * cin
    L.zk_set_option(9, 0)
    print(f"{args.op}{' (no y)' if args.no_y else ''} {shape} b{B} v{args.variant}: "
          f"{us:.1f} us/call "
          f"({flops / us / 1e9:.3f} PF/s)",
          flush=True)


if __name__ == "__main__":
    main()
