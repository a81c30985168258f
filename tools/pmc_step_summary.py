"""Per-kernel PMC summary of a training step from three rocprofv3 --pmc runs
(scripts/gpu.sh pmc): pass 1 SQ counters (MFMA busy, LDS), pass 2
FETCH_SIZE, pass 3 WRITE_SIZE.  Only the last ``--last`` dispatches of each
kernel name are kept (the timed steps, not warmup/MIOpen find trials).

    python tools/pmc_step_summary.py <pmc1.csv> <pmc2.csv> <pmc3.csv> [--top 20]

Columns: total us and calls (pass 1's timestamps; counter collection
serialises the kernels, so durations are per kernel without overlap), MFMA
busy = SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES (summed over XCDs/SEs, a
ratio for comparing kernels, not an absolute utilisation), LDS bank-conflict
cycles per LDS instruction, HBM read (2 x FETCH_SIZE, see MI355X_MICROARCH.md
"FETCH_SIZE reports half the bytes") and write bytes, and the bandwidth they
imply over the kernel's duration.
"""

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)[:72]


def load(path):
    per = defaultdict(dict)
    info = {}
    for r in csv.DictReader(open(path)):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] = float(r["Counter_Value"])
        info[k] = (short(r["Kernel_Name"]),
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per, info


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs=3)
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--frac", type=float, default=0.5,
                    help="keep the last fraction of dispatches (timed steps)")
    a = ap.parse_args()
    passes = [load(p) for p in a.csvs]
    agg = defaultdict(lambda: defaultdict(float))
    for pi, (per, info) in enumerate(passes):
        ids = sorted(per)
        ids = ids[int(len(ids) * (1 - a.frac)):]
        for k in ids:
            name, us = info[k]
            g = agg[name]
            if pi == 0:
                g["us"] += us
                g["calls"] += 1
                for c in ("SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT",
                          "SQ_INSTS_LDS"):
                    g[c] += per[k].get(c, 0.0)
            elif pi == 1:
                g["rd_bytes"] += 2 * per[k].get("FETCH_SIZE", 0.0) * 1024
                g["rd_us"] += us
            else:
                g["wr_bytes"] += per[k].get("WRITE_SIZE", 0.0) * 1024
                g["wr_us"] += us
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["us"])
    total = sum(g["us"] for _, g in rows)
    print(f"kernel time in the window (serialised): {total / 1e3:.2f} ms\n")
    print("| us | calls | MFMA busy | LDS confl/inst | HBM rd MB | HBM wr MB | TB/s | kernel |")
    print("|---:|---:|---:|---:|---:|---:|---:|---|")
    for name, g in rows[:a.top]:
        mf = g["SQ_VALU_MFMA_BUSY_CYCLES"] / g["SQ_BUSY_CYCLES"] if g["SQ_BUSY_CYCLES"] else 0
        lds = g["SQ_LDS_BANK_CONFLICT"] / g["SQ_INSTS_LDS"] if g["SQ_INSTS_LDS"] else 0
        bw_rd = g["rd_bytes"] / (g["rd_us"] * 1e-6) / 1e12 if g["rd_us"] else 0
        bw_wr = g["wr_bytes"] / (g["wr_us"] * 1e-6) / 1e12 if g["wr_us"] else 0
        print(f"| {g['us']:.0f} | {g['calls']:.0f} | {mf:.2f} | {lds:.2f} | "
              f"{g['rd_bytes'] / 1e6:.1f} | {g['wr_bytes'] / 1e6:.1f} | {bw_rd + bw_wr:.2f} | "
              f"`{name}` |")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
