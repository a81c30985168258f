"""Build the native library ``zookeeper_amd/_zkamd.so`` with hipcc for gfx950.

    python -m zookeeper_amd.csrc.build [--force] [-j N]

* ``kernels/*.hip`` are compiled with ``hipcc --offload-arch=gfx950 -O3``
  (device + host code, wave64 CDNA4 only);
* ``runtime/*.cpp`` are host-only C++17 (compiled by hipcc too, so one
  toolchain links everything);
* objects are cached under ``build/zkamd/`` and rebuilt when the CONTENT of
  the source, any header or the compile command changes (a sha256 key next
  to each object; modification times are not trusted -- a copied tree keeps
  stale mtimes); compilation runs in parallel;
* the library embeds ``source_digest()`` -- a sha256 over every kernel /
  runtime source and header -- as ``const char* zk_build_digest()``; the
  loader (``ops/_native.py``) refuses a library whose digest differs from
  the tree it sits in;
* the library links against ``libamdhip64.so.7`` — loaded after ``import
  torch`` it binds to torch's already-loaded HIP runtime (same SONAME).

The library is built in-tree so it travels with the repository snapshot to
the GPU boxes (it is git-ignored).  No hipify, no CUDA headers, no
multi-arch fat binaries.
"""

from __future__ import annotations

import argparse
import glob
import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional

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


def _hash_files(paths: List[str], h: Optional["hashlib._Hash"] = None) -> "hashlib._Hash":
    h = h or hashlib.sha256()
    for p in sorted(paths, key=lambda q: os.path.relpath(q, HERE)):
        h.update(os.path.relpath(p, HERE).replace(os.sep, "/").encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h


def source_digest() -> Optional[str]:
    """sha256 over the kernel / runtime sources and headers (None: no sources,
    e.g. an installed package without ``csrc``)."""
    files = sources() + headers()
    if not files:
        return None
    return _hash_files(files).hexdigest()


def _key_ok(path: str, key: str) -> bool:
    try:
        with open(path + ".key") as f:
            return f.read() == key and os.path.exists(path)
    except OSError:
        return False


def _write_key(path: str, key: str) -> None:
    with open(path + ".key", "w") as f:
        f.write(key)


# Per-file code-generation flags.  wgrad_rows.hip: keep the MFMA accumulators
# in VGPRs (the default AGPR form made the compiler copy all 144 loop-carried
# accumulator registers AGPR <-> VGPR on every step of the main loop).
FILE_FLAGS = {
    "wgrad_rows.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}


def _compile_cmd(src: str, obj: str, extra: List[str]) -> List[str]:
    cmd = [hipcc(), "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
           "-Wno-unused-function", "-Wno-unused-variable", "-Wno-unused-result"]
    if src.endswith(".hip"):
        cmd += [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"]
    else:
        # host C++: the HIP runtime API headers (no device code, no offload)
        rocm = os.path.dirname(os.path.dirname(os.path.realpath(hipcc())))
        cmd += ["-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(rocm, "include")]
    return cmd + FILE_FLAGS.get(os.path.basename(src), []) + extra + ["-c", src, "-o", obj]


def compile_one(src: str, extra: List[str], hdr_digest: str = "") -> str:
    obj = _obj_path(src)
    cmd = _compile_cmd(src, obj, extra)
    key = _hash_files([src], hashlib.sha256(("\0".join(cmd[1:]) + hdr_digest).encode())).hexdigest()
    if _key_ok(obj, key):
        return obj
    os.makedirs(OBJ_DIR, exist_ok=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    _write_key(obj, key)
    return obj


def _digest_object(digest: str) -> str:
    """A host object exporting ``zk_build_digest`` (the only generated source)."""
    os.makedirs(OBJ_DIR, exist_ok=True)
    src = os.path.join(OBJ_DIR, "build_digest.cpp")
    text = ('extern "C" __attribute__((visibility("default"))) const char* zk_build_digest() '
            f'{{ return "{digest}"; }}\n')
    old = None
    if os.path.exists(src):
        with open(src) as f:
            old = f.read()
    if old != text:
        with open(src, "w") as f:
            f.write(text)
    return compile_one(src, [])


def build(force: bool = False, jobs: int = 0, verbose: bool = True) -> str:
    srcs = sources()
    if force:
        shutil.rmtree(OBJ_DIR, ignore_errors=True)
    digest = source_digest()
    hdr = _hash_files(headers()).hexdigest()
    jobs = jobs or min(8, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: compile_one(s, [], hdr), srcs))
    objs.append(_digest_object(digest))
    link_key = _hash_files(objs).hexdigest()
    if force or not _key_ok(OUT, link_key):
        tmp = OUT + ".tmp"
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp, *objs,
               "-lpthread", "-ldl"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, OUT)
        _write_key(OUT, link_key)
    if verbose:
        print(f"[zkamd] built {OUT} from {len(srcs)} sources (digest {digest[:16]})",
              file=sys.stderr)
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
