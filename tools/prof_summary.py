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


# (substring, family), first match wins.  Kernel names are matched on the
# demangled name; every kernel of csrc/kernels has a rule here
# (tests/test_prof_summary.py checks a fixture of every name in a step).
FAMILY_RULES = [
    ("stem_", "stem (fused 7x7 conv / BN / pool)"),
    ("wgrad_rows_kernel", "weight gradient (MFMA)"),
    ("wr_pad_init_kernel", "weight gradient (MFMA)"),
    ("wgrad_deep_kernel", "weight gradient (MFMA)"),
    ("igemm_wgrad", "weight gradient (MFMA)"),
    ("wgrad_reduce", "weight gradient (MFMA)"),
    ("smallk_wgrad", "weight gradient (MFMA)"),
    ("band_wgrad", "weight gradient (MFMA)"),
    ("bconv_wgrad", "weight gradient (MFMA)"),
    ("dgrad_deep_kernel", "data gradient (MFMA)"),
    ("conv3rw_dgrad", "data gradient (MFMA)"),
    ("bconv_dgrad", "data gradient (MFMA)"),
    ("igemm_conv3_kernel<true", "conv forward (MFMA; binary ±1 or float)"),
    ("bfwd", "conv forward (MFMA; binary ±1 or float)"),
    ("igemm_conv_kernel<true", "conv forward (MFMA; binary ±1 or float)"),
    ("bconv_fwd", "conv forward (MFMA; binary ±1 or float)"),
    # FWD=false: the data gradients and the float 1x1 forward GEMMs
    ("igemm_conv", "data gradient / float 1x1 forward (MFMA)"),
    ("smallk_fwd", "small-K / band conv forward (MFMA)"),
    ("band_fwd", "small-K / band conv forward (MFMA)"),
    ("sk_pack", "sign / weight packing"),
    ("bn_", "batch norm (apply / stats / backward)"),
    ("ste_combine", "batch norm (apply / stats / backward)"),
    ("reduce_partials", "batch norm (apply / stats / backward)"),
    ("partials_colsum", "batch norm (apply / stats / backward)"),
    ("dw_", "depthwise conv"),
    ("pool", "pooling"),
    ("gap_", "classifier head (GAP + dense)"),
    ("head_", "classifier head (GAP + dense)"),
    ("sgemm", "classifier head (GAP + dense)"),
    ("weight_pack", "sign / weight packing"),
    ("sign_pack", "sign / weight packing"),
    ("unpack_sign", "sign / weight packing"),
    ("weight_images", "optimizer"),
    ("adam", "optimizer"),
    ("sgd", "optimizer"),
    ("xent", "softmax cross-entropy"),
    ("normalize_flip", "input preprocessing"),
    # HIP runtime blit kernels: copies to / from pinned host memory and
    # memsets (hipMemcpyAsync / hipMemsetAsync)
    ("__amd_rocclr_", "HIP runtime copy / fill"),
]


def family(name: str) -> str:
    n = name
    for key, fam in FAMILY_RULES:
        if key in n[:120]:
            return fam
    if n.startswith("Cijk") or "gtc" in n or "MIOpen" in n or "ck::" in n or "SubTensor" in n:
        return "library (hipBLASLt / MIOpen)"
    if "at::native" in n:
        return "torch elementwise / fill"
    return "other"


def is_step_end(name: str) -> bool:
    """The fused optimizer launch that ends every training step."""
    return "adam_chunks" in name or "sgd_chunks" in name


def refamily_md(path: str) -> str:
    """A family table recomputed with :data:`FAMILY_RULES` from the per-kernel
    rows (``| ms/step | calls/step | avg us | `name` |``) of a kept profile
    summary: for summaries written before the rules covered every kernel."""
    fam = collections.Counter()
    listed = 0.0
    total = None
    for line in open(path):
        if line.startswith("Total kernel time per step:"):
            total = float(line.split(":")[1].split()[0])
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        if len(cells) == 4 and cells[3].startswith("`"):
            try:
                ms = float(cells[0])
            except ValueError:
                continue
            fam[family(cells[3].strip("`"))] += ms
            listed += ms
    out = ["| ms/step | share | family |", "|---:|---:|---|"]
    total = total or listed
    for k, v in fam.most_common():
        out.append(f"| {v:.3f} | {100 * v / total:.1f}% | {k} |")
    if total > listed + 1e-9:
        out.append(f"| {total - listed:.3f} | {100 * (total - listed) / total:.1f}% | "
                   "kernels below the listed rows |")
    return "\n".join(out)


def _trace_window(trace, k: int):
    """Aggregate a kernel trace over the last ``k`` optimizer-delimited steps
    into rows shaped like ``run_kernel_stats.csv``."""
    opt = sorted(int(r["End_Timestamp"]) for r in trace if is_step_end(r["Kernel_Name"]))
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
