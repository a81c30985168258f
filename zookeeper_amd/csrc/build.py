"""Build the native library ``zookeeper_amd/_zkamd.so`` with hipcc for gfx950.

    python -m zookeeper_amd.csrc.build [--force] [-j N]

* ``kernels/*.hip`` are compiled with ``hipcc --offload-arch=gfx950 -O3``
  (device + host code, wave64 CDNA4 only);
* ``runtime/*.cpp`` are host-only C++17 (compiled by hipcc too, so one
  toolchain links everything);
* objects are cached under ``build/zkamd/`` and rebuilt when the source or
  any header is newer; compilation runs in parallel;
* the library links against ``libamdhip64.so.7`` — loaded after ``import
  torch`` it binds to torch's already-loaded HIP runtime (same SONAME).

The library is built in-tree so it travels with the repository snapshot to
the GPU boxes (it is git-ignored).  No hipify, no CUDA headers, no
multi-arch fat binaries.
"""

from __future__ import annotations

import argparse
import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from typing import List

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
OUT = os.path.join(PKG, "_zkamd.so")
OBJ_DIR = os.path.join(ROOT, "build", "zkamd")
ARCH = os.environ.get("ZK_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required)")


def sources() -> List[str]:
    return sorted(glob.glob(os.path.join(HERE, "kernels", "*.hip"))) + sorted(
        glob.glob(os.path.join(HERE, "runtime", "*.cpp"))
    )


def headers() -> List[str]:
    return glob.glob(os.path.join(HERE, "**", "*.h"), recursive=True)


def _obj_path(src: str) -> str:
    rel = os.path.relpath(src, HERE).replace(os.sep, "_")
    return os.path.join(OBJ_DIR, rel + ".o")


def _stale(target: str, deps: List[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def compile_one(src: str, extra: List[str]) -> str:
    obj = _obj_path(src)
    if not _stale(obj, [src] + headers()):
        return obj
    os.makedirs(OBJ_DIR, exist_ok=True)
    cmd = [hipcc(), "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
           "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-result"]
    if src.endswith(".hip"):
        cmd += [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
    else:
        cmd += ["-x", "c++"]
    cmd += extra + ["-c", src, "-o", obj]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return obj


def build(force: bool = False, jobs: int = 0, verbose: bool = True) -> str:
    srcs = sources()
    if force:
        shutil.rmtree(OBJ_DIR, ignore_errors=True)
    jobs = jobs or min(8, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: compile_one(s, []), srcs))
    if _stale(OUT, objs) or force:
        tmp = OUT + ".tmp"
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp, *objs,
               "-lpthread"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, OUT)
    if verbose:
        print(f"[zkamd] built {OUT} from {len(srcs)} sources", file=sys.stderr)
    return OUT


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    args = ap.parse_args()
    build(args.force, args.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
