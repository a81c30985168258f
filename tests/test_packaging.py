"""Packaging checks (reference: setup.py:1-54 and zookeeper/test_version.py):
the distribution's version equals the package's, and the package data globs
cover every native source so an sdist can rebuild the gfx950 library."""

import glob
import os
import subprocess
import sys

import zookeeper_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_setup_version_matches_package():
    out = subprocess.run([sys.executable, "setup.py", "--version"], cwd=ROOT,
                         env=dict(os.environ, ZK_SKIP_NATIVE="1"), capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == zookeeper_amd.__version__


def test_package_data_covers_native_sources():
    from zookeeper_amd.csrc.build import sources

    pkg = os.path.join(ROOT, "zookeeper_amd")
    patterns = ["csrc/*.h", "csrc/kernels/*.hip", "csrc/kernels/*.h", "csrc/runtime/*.cpp"]
    covered = {os.path.abspath(p) for pat in patterns for p in glob.glob(os.path.join(pkg, pat))}
    headers = glob.glob(os.path.join(pkg, "csrc", "**", "*.h"), recursive=True)
    for src in list(sources()) + headers:
        assert os.path.abspath(src) in covered, src


def test_config_layer_microbenchmark_runs(tmp_path):
    """tools/bench_config.py (profiles/config_layer_overheads.md) keeps working."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "cfg.json"
    subprocess.run([sys.executable, os.path.join(root, "tools", "bench_config.py"),
                    "--json", str(out)], check=True, capture_output=True, timeout=300)
    res = json.loads(out.read_text())
    for key in ("import_ms", "configure_tree_plus_first_touches_us", "cached_field_access_us",
                "first_field_access_inherited_us", "cached_factory_field_access_us"):
        assert res[key] > 0, key
