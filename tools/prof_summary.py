"""Summarise a ``rocprofv3 --kernel-trace --stats`` run as a markdown table
(per-step kernel time, grouped by kernel family).

    python tools/prof_summary.py gpurun_out/r1ac_prof/run_kernel_stats.csv \\
        --steps 13 --title "BinaryResNet-E18 ..." --note "bench: ..." > profiles/x.md

With ``--last K`` the argument is a ``run_kernel_trace.csv`` instead and only
the last K *steady-state* steps are counted: the window runs from the end of
the (K+1)-th-from-last optimizer launch to the end of the last one, so one-time
work (MIOpen find trials, first-call packing) in the warmup steps drops out.
"""

import argparse
import collections
import csv


def family(name: str) -> str:
    n = name
    if "stem_" in n:
        return "stem (fused 7x7 conv / BN / pool)"
    if "igemm_wgrad" in n or "wgrad_reduce" in n:
        return "binary/1x1 conv weight gradient (MFMA)"
    if "igemm_conv3_kernel<true" in n or "igemm_conv_kernel<true" in n:
        return "binary conv forward (MFMA)"
    if "igemm_conv" in n:
        return "conv data gradient / 1x1 forward (MFMA)"
    if "bn_" in n[:80]:
        return "batch norm (apply / stats / backward)"
    if "dw_" in n[:60]:
        return "depthwise conv"
    if "pool" in n[:60]:
        return "pooling"
    if "weight_pack" in n or "sign_pack" in n:
        return "sign / weight packing"
    if "adam" in n or "sgd" in n:
        return "optimizer"
    if "xent" in n:
        return "softmax cross-entropy"
    if n.startswith("Cijk") or "gtc" in n or "MIOpen" in n or "ck::" in n or "SubTensor" in n:
        return "library (hipBLASLt / MIOpen)"
    if "at::native" in n:
        return "torch elementwise / fill"
    return "other"


def _trace_window(trace, k: int):
    """Aggregate a kernel trace over the last ``k`` optimizer-delimited steps
    into rows shaped like ``run_kernel_stats.csv``."""
    opt = sorted(int(r["End_Timestamp"]) for r in trace
                 if family(r["Kernel_Name"]) == "optimizer")
    if len(opt) < k + 1:
        raise SystemExit(f"trace has {len(opt)} optimizer launches, need {k + 1}")
    lo, hi = opt[-k - 1], opt[-1]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in trace:
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if lo < t0 and t1 <= hi:
            agg[r["Kernel_Name"]][0] += 1
            agg[r["Kernel_Name"]][1] += t1 - t0
    rows = [{"Name": n, "Calls": c, "TotalDurationNs": d, "AverageNs": d / c}
            for n, (c, d) in agg.items()]
    rows.sort(key=lambda r: -r["TotalDurationNs"])
    return rows


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=0, help="profiled steps (warmup + timed)")
    ap.add_argument("--title", default="kernel profile")
    ap.add_argument("--note", default="")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--last", type=int, default=0,
                    help="csv is a kernel trace: count only the last K steps")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    if a.last:
        rows = _trace_window(rows, a.last)
        a.steps = a.last
    elif a.steps <= 0:
        ap.error("--steps is required for a run_kernel_stats.csv")
    per = lambda r: float(r["TotalDurationNs"]) / a.steps / 1e6  # noqa: E731
    total = sum(per(r) for r in rows)
    print(f"# {a.title}\n")
    if a.note:
        print(a.note + "\n")
    print(f"Total kernel time per step: {total:.2f} ms\n")
    fam = collections.Counter()
    for r in rows:
        fam[family(r["Name"])] += per(r)
    print("| ms/step | share | family |\n|---:|---:|---|")
    for k, v in fam.most_common():
        print(f"| {v:.3f} | {100 * v / total:.1f}% | {k} |")
    print(f"\n| ms/step | calls/step | avg us | kernel |\n|---:|---:|---:|---|")
    for r in rows[:a.top]:
        print(f"| {per(r):.3f} | {int(r['Calls']) / a.steps:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | `{r['Name'][:110]}` |")


if __name__ == "__main__":
    main()
