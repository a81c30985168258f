"""Host-side native runtime under the sanitizers: the threaded
row gather of ``csrc/runtime/host_ring.cpp`` built with AddressSanitizer +
UndefinedBehaviorSanitizer and, separately, ThreadSanitizer (sanitizer
runtimes linked statically), driven by ``tests/native/host_ring_check.cpp``.
Host code only (no GPU sanitizers on this pool); skipped when the compiler or
the sanitizer runtime is missing."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "zookeeper_amd", "csrc", "runtime", "host_ring.cpp"),
       os.path.join(ROOT, "tests", "native", "host_ring_check.cpp")]


def _build_and_run(tmp_path, flags, env_extra):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "host_ring_check")
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread", *flags,
           *SRC, "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0:
        pytest.skip(f"sanitizer build unavailable: {b.stderr[-300:]}")
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_ring_check: ok" in r.stdout


def test_host_ring_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                              "-static-libasan", "-static-libubsan"],
                   {"ASAN_OPTIONS": "detect_leaks=1"})


def test_host_ring_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread", "-static-libtsan"],
                   {"TSAN_OPTIONS": "halt_on_error=1"})
