"""Per-kernel resource table (VGPRs, AGPRs, spills, occupancy) of one HIP
source, from hipcc's kernel-resource-usage remarks (gfx950).

    python tools/kres.py zookeeper_amd/csrc/kernels/wgrad_rows.hip [name-filter]
"""
import re
import subprocess
import sys
import tempfile
import os

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, here)


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    from zookeeper_amd.csrc.build import FILE_FLAGS  # per-file flags of the real build
    flags = FILE_FLAGS.get(os.path.basename(src), [])
    csrc = os.path.join(here, "zookeeper_amd", "csrc")
    with tempfile.TemporaryDirectory() as td:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
               "-munsafe-fp-atomics", *flags, "-c", "-I" + csrc, "-I" + os.path.join(csrc, "kernels"),
               src, "-o", os.path.join(td, "o.o"), "-Rpass-analysis=kernel-resource-usage"]
        out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    keys = ["VGPRs", "AGPRs", "SGPRs Spill", "VGPRs Spill", "ScratchSize [bytes/lane]",
            "Occupancy [waves/SIMD]"]
    print("kernel".ljust(60), *[k.split(" [")[0][:11].rjust(11) for k in keys])
    for r in rows:
        if filt in r["name"]:
            print(r["name"][-60:].ljust(60), *[str(r.get(k, "-")).rjust(11) for k in keys])


if __name__ == "__main__":
    main()
