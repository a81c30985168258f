"""Instruction mix of the hottest MFMA basic block of each kernel in a hipcc
--save-temps gfx950 assembly file.

    python tools/isa_loop.py <file.s> [symbol-substring ...]
"""
import re
import sys
from collections import Counter


def main():
    s = open(sys.argv[1]).read()
    names = re.findall(r"^(_Z\S+):", s, re.M)
    filt = sys.argv[2:]
    for nm in names:
        if filt and not any(f in nm for f in filt):
            continue
        i = s.index(nm + ":")
        j = s.find(".Lfunc_end", i)
        body = s[i:j]
        parts = re.split(r"\n(\.LBB\d+_\d+):", body)
        best = None
        for k in range(1, len(parts), 2):
            n = parts[k + 1].count("v_mfma")
            if n and (best is None or n > best[1]):
                best = (parts[k], n, parts[k + 1])
        if best is None:
            continue
        lab, n, b = best
        ins = [ln.strip().split()[0] for ln in b.splitlines()
               if ln.strip() and not ln.strip().startswith((".", ";", "/"))]
        c = Counter(ins)
        grp = lambda f: sum(v for k, v in c.items() if f(k))
        print(f"{nm[-40:]:40s} {lab:10s} mfma {n:3d} total {len(ins):4d} "
              f"accvgpr {grp(lambda k: 'accvgpr' in k):3d} "
              f"valu {grp(lambda k: k.startswith('v_') and 'mfma' not in k):4d} "
              f"ds {grp(lambda k: k.startswith('ds_')):3d} "
              f"vmem {grp(lambda k: k.startswith(('global_', 'buffer_'))):3d} "
              f"salu {grp(lambda k: k.startswith('s_')):4d}")


if __name__ == "__main__":
    main()
