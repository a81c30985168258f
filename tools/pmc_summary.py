"""Summarise rocprofv3 --pmc CSVs: per (kernel, grid) mean of each counter."""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", ""))
    return name.replace("void ", "")[:60]


def load(paths, pattern):
    d = defaultdict(lambda: defaultdict(list))
    meta = {}
    for p in paths:
        per = defaultdict(dict)
        info = {}
        for r in csv.DictReader(open(p)):
            if not re.search(pattern, r["Kernel_Name"]):
                continue
            key = (r["Dispatch_Id"])
            per[key][r["Counter_Name"]] = float(r["Counter_Value"])
            info[key] = (short(r["Kernel_Name"]), int(r["Grid_Size"]), r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"],
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        for k, cs in per.items():
            name, grid, vg, ag, lds, us = info[k]
            kk = (name, grid)
            meta[kk] = (vg, ag, lds)
            for c, v in cs.items():
                d[kk][c].append(v)
            d[kk]["us"].append(us)
    return d, meta


if __name__ == "__main__":
    pattern = sys.argv[1]
    d, meta = load(sys.argv[2:], pattern)
    for kk in sorted(d):
        cs = d[kk]
        print(kk[0], "grid", kk[1], "vgpr/agpr/lds", meta[kk])
        print("   " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())))
