"""Build provenance: the native library carries a digest of the sources it
was built from, the loader refuses a library that does not match the tree,
and ``backend="auto"`` on a GPU raises instead of falling back to the
library (MIOpen / hipBLASLt) path when the native library is unusable.

VERDICT r3 "What's weak" 4 and 6: a stale ``.so`` pushed with the tree, or a
failed load, must not be able to produce a headline number silently."""

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "zookeeper_amd")
LIB = os.path.join(PKG, "_zkamd.so")

_PROBE = ("import torch, json; from zookeeper_amd.ops import _native as n; "
          "print(json.dumps([n.available(), n.load_error()]))")


def _probe(root):
    import json

    env = dict(os.environ, PYTHONPATH=root, ZK_NATIVE="1")
    res = subprocess.run([sys.executable, "-c", _PROBE], cwd=root, env=env, capture_output=True,
                         text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    return json.loads(res.stdout.strip().splitlines()[-1])


@pytest.mark.timeout(600)
def test_touched_kernel_source_refuses_the_library_until_rebuilt(tmp_path):
    if not os.path.exists(LIB) or shutil.which("hipcc") is None and not os.path.exists(
            "/opt/rocm/bin/hipcc"):
        pytest.skip("needs the built library and hipcc")
    root = str(tmp_path)
    shutil.copytree(PKG, os.path.join(root, "zookeeper_amd"),
                    ignore=shutil.ignore_patterns("__pycache__"))
    objs = os.path.join(ROOT, "build", "zkamd")
    if os.path.isdir(objs):  # object cache: only the touched file recompiles
        shutil.copytree(objs, os.path.join(root, "build", "zkamd"))
    ok, err = _probe(root)
    assert ok, err  # the copy as made loads

    src = os.path.join(root, "zookeeper_amd", "csrc", "kernels", "preprocess.hip")
    with open(src, "a") as f:
        f.write("\n// touched by test_build_provenance\n")
    ok, err = _probe(root)
    assert not ok and "stale" in err, err

    env = dict(os.environ, PYTHONPATH=root)
    res = subprocess.run([sys.executable, "-m", "zookeeper_amd.csrc.build"], cwd=root, env=env,
                         capture_output=True, text=True, timeout=540)
    assert res.returncode == 0, res.stderr[-3000:]
    ok, err = _probe(root)
    assert ok, err


def test_source_digest_covers_kernels_runtime_and_headers():
    from zookeeper_amd.csrc import build

    files = {os.path.relpath(p, build.HERE) for p in build.sources() + build.headers()}
    assert any(f.startswith("kernels") and f.endswith(".hip") for f in files)
    assert any(f.startswith("runtime") and f.endswith(".cpp") for f in files)
    assert "common.h" in files and os.path.join("kernels", "mfma_common.h") in files
    d = build.source_digest()
    assert isinstance(d, str) and len(d) == 64


def test_auto_backend_raises_on_a_gpu_without_the_native_library(monkeypatch):
    import torch

    from zookeeper_amd import configure
    from zookeeper_amd.models import BinaryResNetE18
    from zookeeper_amd.ops import _native

    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(_native, "_tried", True)
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "_load_error", "zookeeper_amd/_zkamd.so not built")
    monkeypatch.delenv("ZK_NATIVE", raising=False)
    m = BinaryResNetE18()
    configure(m, {"input_shape": (32, 32, 3), "dataset": _dataset()})
    with pytest.raises(RuntimeError, match="native library"):
        m.resolved_backend()
    # deliberate opt-out: the PyTorch path, no error
    monkeypatch.setenv("ZK_NATIVE", "0")
    assert m.resolved_backend() == "torch"
    # and with no GPU at all, auto is the oracle path
    monkeypatch.delenv("ZK_NATIVE")
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    assert m.resolved_backend() == "torch"


def _dataset():
    from zookeeper_amd.data import SyntheticCIFAR10

    return SyntheticCIFAR10()
