"""The ctypes signature table must match the C ABI declared in the HIP/C++
sources (argument counts and pointer/integer/float kinds), checked on CPU by
parsing every ``ZK_EXPORT`` / ``extern "C"`` definition."""

import glob
import os
import re

from zookeeper_amd.ops import _signatures

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "zookeeper_amd", "csrc")

_DEF = re.compile(
    r'(?:ZK_EXPORT|extern\s+"C"\s+__attribute__\(\(visibility\("default"\)\)\))\s+'
    r"(?:int|long long)\s+(zk_\w+)\s*\(([^)]*)\)", re.S)


def _kind(param: str) -> str:
    p = " ".join(param.split())
    if "*" in p or "hipStream_t" in p:
        return "P"
    if "double" in p:
        return "D"
    if "float" in p:
        return "F"
    if "long long" in p or "int64_t" in p:
        return "I64"
    return "I32"


def _ctypes_kind(t) -> str:
    import ctypes as C

    if t in (C.c_void_p,) or getattr(t, "_type_", None) is not None and t not in (
            C.c_int, C.c_int64, C.c_float, C.c_double, C.c_uint64):
        return "P"
    return {C.c_int: "I32", C.c_int64: "I64", C.c_uint64: "I64", C.c_float: "F",
            C.c_double: "D"}[t]


def parse_exports():
    out = {}
    for f in glob.glob(os.path.join(ROOT, "**", "*.hip"), recursive=True) + glob.glob(
            os.path.join(ROOT, "**", "*.cpp"), recursive=True):
        src = open(f).read()
        for name, params in _DEF.findall(src):
            ps = [p for p in params.split(",") if p.strip()]
            out[name] = [_kind(p) for p in ps]
    return out


def test_every_export_has_a_matching_signature():
    exports = parse_exports()
    assert exports, "no exports parsed"
    for name, kinds in exports.items():
        assert name in _signatures.SIGNATURES, f"{name} missing from _signatures"
        _, argtypes = _signatures.SIGNATURES[name]
        got = [_ctypes_kind(a) for a in argtypes]
        # unsigned long long seeds are passed as c_uint64 (kind I64)
        want = ["I64" if k == "I64" else k for k in kinds]
        assert got == want, f"{name}: ctypes {got} != C {want}"
    for name in _signatures.SIGNATURES:
        if name in GENERATED:
            continue
        assert name in exports, f"{name} declared in _signatures but not exported"


# exports the build generates (csrc/build.py), not written in the sources
GENERATED = {"zk_build_digest"}


def test_built_library_carries_the_tree_digest():
    """The loaded library's embedded digest is the digest of the sources
    next to it (``_native._load`` refuses the library otherwise)."""
    import pytest

    from zookeeper_amd.csrc import build
    from zookeeper_amd.ops import _native

    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("native library not built")
    assert _native.available(), _native.load_error()
    assert _native.build_digest() == build.source_digest()
