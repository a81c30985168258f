"""Standalone check and timing of the row-streaming 3x3 weight gradient
(``zk_wgrad_rows``, csrc/kernels/wgrad_rows.hip) against the previous default
kernels (``zk_igemm_wgrad``: conv3 tiles + slab reduce) and an fp32 oracle.

    python tools/wgrad_lab.py [--batch 1536] [--shapes 56,64,64/28,128,128] [--reps 20]

Per shape (H=W, Cin, Cout): max relative error of each kernel against the fp32
oracle at --check-batch, the bitwise run-to-run equality of the new kernel,
the new-vs-old relative difference at --batch, and interleaved timings
(median us over --rounds rounds of --reps launches each).
"""

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def make(B, H, Cin, Cout, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(B, H, H, Cin, device=dev, generator=g).to(torch.bfloat16)
    x = torch.where(x == 0, torch.zeros_like(x), x)  # no -0 (producers never store it)
    sx = torch.where(x >= 0, 1.0, -1.0).to(torch.bfloat16)
    dy = torch.randn(B, H, H, Cout, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.rand(Cout, 3, 3, Cin, device=dev, generator=g) * 2.6 - 1.3).contiguous()
    return x, sx, dy, w


def fp4(sx):
    """e2m1 sign image (channel 2j in the low nibble of byte j)."""
    code = torch.where(sx.float() >= 0, 2, 10).to(torch.uint8)
    return (code[..., 0::2] | (code[..., 1::2] << 4)).contiguous()


def oracle(sx, dy, w, pad_ones, clip):
    xp = torch.nn.functional.pad(sx.float().permute(0, 3, 1, 2), (1, 1, 1, 1),
                                 value=1.0 if pad_ones else 0.0)
    gw = torch.nn.grad.conv2d_weight(xp, (w.shape[0], w.shape[3], 3, 3),
                                     dy.float().permute(0, 3, 1, 2), padding=0)
    return gw.permute(0, 2, 3, 1) * (w.abs() <= clip).float()


class Rows:
    def __init__(self, L, B, H, Cin, Cout, tb, dev):
        import ctypes
        sb, cb = ctypes.c_int64(0), ctypes.c_int64(0)
        rc = L.zk_wgrad_rows_plan(B, H, H, Cin, Cout, tb, ctypes.byref(sb), ctypes.byref(cb))
        if rc != 0:
            raise RuntimeError("shape not supported by zk_wgrad_rows")
        self.slab = torch.empty(max(sb.value // 4, 1), dtype=torch.float32, device=dev)
        self.cnt = torch.zeros(max(cb.value // 4, 1), dtype=torch.int32, device=dev)
        self.sb, self.cb, self.tb = sb.value, cb.value, tb
        self.L, self.geo = L, (B, H, H, Cin, Cout)

    def __call__(self, dy, s, w, dw, sign, st):
        B, H, W, Cin, Cout = self.geo
        rc = self.L.zk_wgrad_rows(dy.data_ptr(), s.data_ptr(), w.data_ptr(), dw.data_ptr(),
                                  self.slab.data_ptr(), self.sb, self.cnt.data_ptr(), self.cb,
                                  B, H, W, Cin, Cout, 1, int(sign), 1.0, self.tb, st)
        if rc:
            raise RuntimeError(f"zk_wgrad_rows rc={rc}")


def old_wgrad(L, dy, sx, w, dw, B, H, Cin, Cout, st, ws_cache={}):
    key = (B, H, Cin, Cout)
    if key not in ws_cache:
        nb = int(L.zk_igemm_wgrad_ws_bytes(B, Cin, H, H, H, H, Cout, 3, 3, 1, 1, 1, 0, -1))
        ws_cache[key] = (torch.empty(max(nb // 4, 1), dtype=torch.float32, device=dw.device), nb)
    ws, nb = ws_cache[key]
    rc = L.zk_igemm_wgrad(dy.data_ptr(), sx.data_ptr(), w.data_ptr(), dw.data_ptr(), B, H, H, Cin,
                          H, H, Cout, 3, 3, 1, 1, 1, 1, 1.0, 0, -1, ws.data_ptr(), nb, st)
    if rc:
        raise RuntimeError(f"zk_igemm_wgrad rc={rc}")


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1536)
    ap.add_argument("--check-batch", type=int, default=24)
    ap.add_argument("--shapes", default="56,64,64/28,128,128")
    ap.add_argument("--tbs", default="256")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--pmc", action="store_true",
                    help="only launch the row kernel (sign mode) --reps times per shape "
                         "(a rocprofv3 --pmc target)")
    args = ap.parse_args()
    from zookeeper_amd.ops._native import lib, stream_ptr

    L = lib()
    dev = torch.device("cuda")
    st = stream_ptr(dev)
    rows = []
    for shp in args.shapes.split("/"):
        H, Cin, Cout = (int(v) for v in shp.replace("x", ",").split(","))
        tbs = [int(t) for t in args.tbs.replace("x", ",").split(",")]
        if args.pmc:
            B = args.batch
            x, sx, dy, w = make(B, H, Cin, Cout, dev, seed=1)
            dw = torch.zeros_like(w)
            k = Rows(L, B, H, Cin, Cout, tbs[0], dev)
            for _ in range(args.reps):
                k(dy, x, w, dw, 1, st)
            torch.cuda.synchronize()
            print(f"pmc target done: {H}x{Cin}x{Cout} b{B} x{args.reps}", flush=True)
            del x, sx, dy, w, dw, k
            continue
        # --- numerics at the check batch
        B = args.check_batch
        x, sx, dy, w = make(B, H, Cin, Cout, dev)
        ref = oracle(sx, dy, w, True, 1.0)
        scale = ref.abs().max().item()
        rec = {"shape": [H, H, Cin, Cout], "check_batch": B}
        sx4 = fp4(sx)
        for tb in tbs + [8, 3]:
            k = Rows(L, B, H, Cin, Cout, tb, dev)
            for sign in (0, 1, 2):
                dw = torch.full_like(w, 0.25)  # accumulates into existing values
                k(dy, (sx, x, sx4)[sign], w, dw, sign, st)
                torch.cuda.synchronize()
                err = ((dw - 0.25 * (w.abs() <= 1.0).float() - 0.25 * (w.abs() > 1.0).float()
                        - ref).abs().max().item()) / scale
                rec[f"rows_tb{tb}_sign{sign}_relerr"] = err
        dw = torch.zeros_like(w)
        old_wgrad(L, dy, sx, w, dw, B, H, Cin, Cout, st)
        torch.cuda.synchronize()
        rec["old_relerr"] = (dw - ref).abs().max().item() / scale
        del x, sx, sx4, dy, w, ref
        # --- full batch: determinism, new vs old, timings
        B = args.batch
        x, sx, dy, w = make(B, H, Cin, Cout, dev, seed=1)
        sx4 = fp4(sx)
        ks = {tb: Rows(L, B, H, Cin, Cout, tb, dev) for tb in tbs}
        outs = []
        for rep in range(2):
            dw = torch.zeros_like(w)
            ks[tbs[0]](dy, x, w, dw, 1, st)
            outs.append(dw)
        dwo = torch.zeros_like(w)
        old_wgrad(L, dy, sx, w, dwo, B, H, Cin, Cout, st)
        torch.cuda.synchronize()
        rec["rows_bitwise_repeat"] = bool(torch.equal(outs[0], outs[1]))
        d4 = torch.zeros_like(w)
        ks[tbs[0]](dy, sx4, w, d4, 2, st)
        torch.cuda.synchronize()
        rec["rows_fp4_equals_sign"] = bool(torch.equal(outs[0], d4))
        del d4
        rec["rows_vs_old_rel"] = ((outs[0] - dwo).abs().max() / dwo.abs().max()).item()
        dw = torch.zeros_like(w)
        fns = {"old": lambda: old_wgrad(L, dy, sx, w, dw, B, H, Cin, Cout, st)}
        for tb in tbs:
            fns[f"rows_tb{tb}_img"] = (lambda k=ks[tb]: k(dy, sx, w, dw, 0, st))
            fns[f"rows_tb{tb}_sign"] = (lambda k=ks[tb]: k(dy, x, w, dw, 1, st))
            fns[f"rows_tb{tb}_fp4"] = (lambda k=ks[tb]: k(dy, sx4, w, dw, 2, st))

        dbg = torch.zeros(4096 * 4 * 8, dtype=torch.int64, device=dev)

        def ablate(mode, k=ks[tbs[0]]):
            L.zk_wgrad_rows_lab(mode, dbg.data_ptr())
            try:
                k(dy, x, w, dw, 1, st)
            finally:
                L.zk_wgrad_rows_lab(0, None)
        fns["rows_loads_only"] = lambda: ablate(1)
        fns["rows_compute_only"] = lambda: ablate(2)
        fns["rows_lds_reads_only"] = lambda: ablate(3)
        fns["rows_mfma_no_s_reads"] = lambda: ablate(4)
        fns["rows_fd4_sign"] = lambda: ablate(6)
        fns["rows_burst_issue_sign"] = lambda: ablate(8)
        times = {n: [] for n in fns}
        for _ in range(args.rounds):
            for n, fn in fns.items():
                times[n].append(timeit(fn, args.reps))
        for n, t in times.items():
            rec[f"{n}_us_med"] = round(statistics.median(t), 1)
            rec[f"{n}_us_min"] = round(min(t), 1)
        if H == 56:
            dbg.zero_()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            ev0.record()
            ablate(7)
            ev1.record()
            torch.cuda.synchronize()
            ends = dbg.view(-1, 8)
            ends = ends[ends[:, 3] > 0]
            # wall_clock64 ticks of the whole launch vs its event time (us):
            # calibrates the tick rate (events add the launch latency)
            span_ticks = float(ends[:, 7].max() - ends[:, 4].min())
            rec["lab7_event_us"] = round(ev0.elapsed_time(ev1) * 1e3, 1)
            rec["wall_clock_mhz_upper"] = round(span_ticks / (ev0.elapsed_time(ev1) * 1e3), 2)
            dbg.zero_()
            ablate(7)
            torch.cuda.synchronize()
            ends = dbg.view(-1, 8)
            ends = ends[ends[:, 3] > 0]
            rec["tree_tail_us"] = round(float((ends[:, 7].max() - ends[:, 5].max()) / 100.0), 1)
            rec["kernel_span_us"] = round(float((ends[:, 7].max() - ends[:, 4].min()) / 100.0), 1)
            dbg.zero_()
            ablate(7)
            torch.cuda.synchronize()
            d = dbg.view(-1, 8)
            d = d[d[:, 3] > 0].double()
            tot = d[:, :3].sum(0)
            rec["cycles_per_step_wait_issue_mma"] = [round(v, 1) for v in
                                                     (tot / d[:, 3].sum()).tolist()]
            # wall clock (100 MHz): kernel span and per-block main-loop spans
            t0 = d[:, 4].min()
            st_ = (d[:, 4] - t0) / 100.0  # us
            en_ = (d[:, 5] - t0) / 100.0
            rec["loop_span_us"] = round(float(en_.max()), 1)
            rec["block_loop_us_min_med_max"] = [round(float(v), 1) for v in
                                                torch.quantile(en_ - st_, torch.tensor(
                                                    [0.0, 0.5, 1.0], dtype=torch.float64,
                                                    device=d.device)).tolist()]
            rec["block_start_us_min_med_max"] = [round(float(v), 1) for v in
                                                 torch.quantile(st_, torch.tensor(
                                                     [0.0, 0.5, 1.0], dtype=torch.float64,
                                                     device=d.device)).tolist()]
            rec["shader_clock_ghz"] = round(float(((d[:, 2] + d[:, 0] + d[:, 1]).sum()) /
                                                  ((en_ - st_).sum() * 1e3)), 3)
        gbytes = (dy.numel() + x.numel()) * 2 / 1e9
        rec["hbm_floor_us_at_6TBs"] = round(gbytes / 6.0e3 * 1e6, 1)
        rows.append(rec)
        print(json.dumps(rec), flush=True)
        del x, sx, sx4, dy, w, dw, dwo, outs, ks
        torch.cuda.empty_cache()
    if args.out:
        with open(args.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
