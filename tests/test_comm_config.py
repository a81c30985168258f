"""The data-parallel communicator set-up (``Runtime`` comm fields ->
``parallel.dist.CommConfig``): per-rank CPU affinity from sysfs, RCCL
channel knobs, high-priority RCCL streams, and the cross-rank bucket-order
check.  CPU only: fake sysfs trees, gloo."""

import os
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _fake_sysfs(tmp_path, gpus):
    """gpus: list of (pci bus, local cpulist); plus one CPU node 0."""
    kfd = tmp_path / "kfd"
    pci = tmp_path / "pci"
    (kfd / "0").mkdir(parents=True)
    (kfd / "0" / "gpu_id").write_text("0\n")
    (kfd / "0" / "properties").write_text("cpu_cores_count 32\n")
    for i, (bus, cpus) in enumerate(gpus):
        n = kfd / str(i + 1)
        n.mkdir()
        (n / "gpu_id").write_text(f"{1000 + i}\n")
        loc = (bus << 8) | (0 << 3) | 0
        (n / "properties").write_text(f"simd_count 1024\ndomain 0\nlocation_id {loc}\n")
        d = pci / f"0000:{bus:02x}:00.0"
        d.mkdir(parents=True)
        (d / "local_cpulist").write_text(cpus + "\n")
    return str(kfd), str(pci)


def test_parse_cpulist():
    from zookeeper_amd.parallel.affinity import parse_cpulist

    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []


def test_rank_cpus_split_numa_local_lists(tmp_path):
    from zookeeper_amd.parallel.affinity import gpu_pci_addresses, rank_cpus

    kfd, pci = _fake_sysfs(tmp_path, [(0x05, "0-15"), (0x15, "0-15"), (0x85, "16-31"),
                                      (0x95, "16-31")])
    assert gpu_pci_addresses(kfd) == ["0000:05:00.0", "0000:15:00.0", "0000:85:00.0",
                                      "0000:95:00.0"]
    allowed = list(range(32))
    kw = dict(env={}, kfd_root=kfd, pci_root=pci, allowed=allowed)
    # four ranks: two per socket, each half of its socket's list
    assert rank_cpus(0, 4, **kw) == list(range(0, 8))
    assert rank_cpus(1, 4, **kw) == list(range(8, 16))
    assert rank_cpus(2, 4, **kw) == list(range(16, 24))
    assert rank_cpus(3, 4, **kw) == list(range(24, 32))
    # one rank: the whole local list
    assert rank_cpus(0, 1, **kw) == list(range(16)) or rank_cpus(0, 1, **kw) == list(range(0, 16))
    # visible-device remap: local rank 0 drives physical GPU 2
    kw2 = dict(kw, env={"HIP_VISIBLE_DEVICES": "2,3"})
    assert rank_cpus(0, 2, **kw2) == list(range(16, 24))
    assert rank_cpus(1, 2, **kw2) == list(range(24, 32))
    # the process may not use those CPUs: nothing to pin
    assert rank_cpus(0, 1, env={}, kfd_root=kfd, pci_root=pci, allowed=[40, 41]) is None
    # UUID-style device lists: unknown mapping, no pinning
    assert rank_cpus(0, 1, env={"HIP_VISIBLE_DEVICES": "GPU-abc"}, kfd_root=kfd,
                     pci_root=pci, allowed=allowed) is None
    # no topology at all
    assert rank_cpus(0, 1, env={}, kfd_root=str(tmp_path / "none"), pci_root=pci,
                     allowed=allowed) is None


def test_rccl_channel_knobs_and_priority_options():
    from zookeeper_amd.parallel.dist import CommConfig, _pg_options, apply_rccl_env

    env = {}
    assert apply_rccl_env(CommConfig(), env) == {}
    got = apply_rccl_env(CommConfig(min_channels=4, max_channels=16), env)
    assert got == {"NCCL_MIN_NCHANNELS": "4", "NCCL_MAX_NCHANNELS": "16"}
    with pytest.raises(ValueError):
        apply_rccl_env(CommConfig(min_channels=8, max_channels=4), {})
    opts = _pg_options("nccl", CommConfig(high_priority=True))
    assert opts is not None and opts.is_high_priority_stream
    assert _pg_options("nccl", CommConfig(high_priority=False)) is None
    assert _pg_options("gloo", CommConfig(high_priority=True)) is None


def test_runtime_comm_fields_map_to_comm_config():
    from zookeeper_amd import configure
    from zookeeper_amd.train.runtime import Runtime

    rt = Runtime()
    configure(rt, {"rccl_max_channels": 8, "cpu_affinity": False, "check_bucket_order": True,
                   "comm_high_priority": False})
    c = rt.comm_config()
    assert (c.max_channels, c.min_channels, c.cpu_affinity, c.check_bucket_order,
            c.high_priority) == (8, 0, False, True, False)
    d = rt.as_dict()
    for k in ("comm_high_priority", "rccl_min_channels", "rccl_max_channels", "cpu_affinity",
              "check_bucket_order"):
        assert k in d
    bad = Runtime()
    with pytest.raises(ValueError):
        configure(bad, {"rccl_min_channels": 8, "rccl_max_channels": 4})


def test_order_hash_is_position_sensitive():
    from zookeeper_amd.parallel.ddp import order_hash

    assert order_hash([0, 1, 2]) != order_hash([1, 0, 2])
    assert order_hash([0, 1, 2]) == order_hash([0, 1, 2])
    assert 0 <= order_hash(list(range(100))) < 2**61


@pytest.mark.timeout(300)
def test_bucket_order_check_two_ranks(tmp_path):
    """gloo, world size 2: the check runs every step with matching orders,
    and flags ranks whose launch orders differ."""
    from zookeeper_amd.parallel.launch import spawn

    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("RANK", None)
    rc = spawn([sys.executable, os.path.join(HERE, "dp_worker.py"), "order", str(tmp_path)], 2,
               env=env)
    assert rc == 0
    r = [torch.load(tmp_path / f"order{i}.pt", weights_only=True) for i in (0, 1)]
    assert r[0]["checks"] == r[1]["checks"] == 3  # one per training step
    assert r[0]["order"] == r[1]["order"] and len(r[0]["order"]) > 1
    assert r[0]["flagged"] and r[1]["flagged"]


def test_native_communicator_binding_on_cpu():
    """The in-tree RCCL binding resolves torch's bundled librccl by path and
    creates unique ids without a GPU (the communicator itself needs one:
    tests/gpu/test_native_comm.py)."""
    from zookeeper_amd.ops import _native
    from zookeeper_amd.parallel import rccl

    if not _native.available():
        pytest.skip(_native.load_error())
    if rccl.rccl_path() is None:
        pytest.skip("torch ships no librccl")
    rccl.load()
    assert _native.lib().zk_comm_loaded() == 1
    a, b = rccl.unique_id(), rccl.unique_id()
    assert len(a) == 128 and a != b
    assert rccl.DTYPES[torch.float32] == 7 and rccl.OPS["sum"] == 0


def test_runtime_comm_backend_field():
    from zookeeper_amd import configure
    from zookeeper_amd.train.runtime import Runtime

    rt = Runtime()
    configure(rt, {"comm_backend": "native"})
    assert rt.comm_config().backend == "native" and rt.as_dict()["comm_backend"] == "native"
    with pytest.raises(ValueError):
        configure(Runtime(), {"comm_backend": "mpi"})
