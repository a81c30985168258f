"""Stream-level timeline of a training step from a rocprofv3 kernel trace.

    python tools/timeline.py gpurun_out/prof_3/run_kernel_trace.csv --last 6

Over the last K optimizer-delimited steps (as ``prof_summary.py --last``)
prints, per step: wall time, time with at least one kernel running (the
union of kernel intervals), idle gaps, and per-stream (queue) busy time, plus
the kernels on the longest stream with the share of their time that overlaps
another stream.  It answers "is the step bound by the compute stream's
critical path, by GPU idle gaps (host / launch latency), or by the total
kernel work?" — the question a per-kernel table cannot.
"""

import argparse
import collections
import csv


def _union(iv):
    iv = sorted(iv)
    tot, cur0, cur1 = 0, None, None
    for a, b in iv:
        if cur1 is None or a > cur1:
            if cur1 is not None:
                tot += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    if cur1 is not None:
        tot += cur1 - cur0
    return tot


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=6)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    with open(a.trace) as f:
        rows = list(csv.DictReader(f))
    sid = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    opt = sorted(int(r["End_Timestamp"]) for r in rows
                 if "adam" in r["Kernel_Name"] or "sgd" in r["Kernel_Name"])
    if len(opt) < a.last + 1:
        raise SystemExit(f"{len(opt)} optimizer launches, need {a.last + 1}")
    lo, hi = opt[-a.last - 1], opt[-1]
    win = [r for r in rows if lo < int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= hi]
    k = a.last
    wall = (hi - lo) / k / 1e6
    allv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in win]
    busy = _union(allv) / k / 1e6
    per = collections.defaultdict(list)
    for r in win:
        per[r[sid]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    print(f"window: {k} steps, wall {wall:.3f} ms/step, GPU busy (union) {busy:.3f} ms/step, "
          f"idle {wall - busy:.3f} ms/step, kernel sum {sum(b - a_ for a_, b in allv) / k / 1e6:.3f}")
    print()
    print("| stream | kernels/step | busy ms/step (union) | share of wall |")
    print("|---|---:|---:|---:|")
    for s, iv in sorted(per.items(), key=lambda kv: -len(kv[1])):
        u = _union([(x, y) for x, y, _ in iv]) / k / 1e6
        print(f"| {s} | {len(iv) / k:.1f} | {u:.3f} | {100 * u / wall:.1f}% |")
    # overlap of each kernel of the main stream with other streams
    main_s = max(per, key=lambda s: len(per[s]))
    others = sorted((x, y) for s, iv in per.items() if s != main_s for x, y, _ in iv)
    agg = collections.defaultdict(lambda: [0, 0, 0])
    for x, y, n in per[main_s]:
        ov = 0
        for ox, oy in others:
            if ox >= y:
                break
            if oy > x:
                ov += min(y, oy) - max(x, ox)
        nm = n.replace("(anonymous namespace)::", "")
        nm = (nm[5:] if nm.startswith("void ") else nm).split("(")[0][:110]
        agg[nm][0] += 1
        agg[nm][1] += y - x
        agg[nm][2] += min(ov, y - x)
    print()
    print(f"main stream {main_s}: kernels by time (overlap = share of the kernel's time "
          f"during which another stream ran)")
    print()
    print("| ms/step | calls/step | overlap | kernel |")
    print("|---:|---:|---:|---|")
    for nm, (c, t, ov) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| {t / k / 1e6:.3f} | {c / k:.1f} | {100 * ov / max(t, 1):.0f}% | `{nm}` |")
    # gaps on the main stream
    iv = sorted((x, y) for x, y, _ in per[main_s])
    gaps = [iv[i + 1][0] - iv[i][1] for i in range(len(iv) - 1) if iv[i + 1][0] > iv[i][1]]
    print()
    print(f"main-stream gaps: {sum(gaps) / k / 1e6:.3f} ms/step over {len(gaps) / k:.0f}/step, "
          f"largest {max(gaps, default=0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
