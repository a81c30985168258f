"""Kernel / schedule switches are typed config (the ``Runtime`` component),
not environment variables: configurable, recorded, pushed into the ops at
``apply()``; GPU counting for launchers reads only env + sysfs."""

import os
import re

import pytest

from zookeeper_amd import configure
from zookeeper_amd.core.component import flatten_config
from zookeeper_amd.ops import options
from zookeeper_amd.parallel.devices import visible_gpu_count, visible_gpu_ids
from zookeeper_amd.train.runtime import Runtime

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _reset():
    options.reset()
    yield
    options.reset()


def test_runtime_defaults_match_kernel_option_defaults():
    rt = Runtime()
    configure(rt, {})
    assert rt.kernel_options() == options.snapshot()


def test_runtime_apply_sets_options():
    rt = Runtime()
    configure(rt, {"bconv_fp4": False, "tile_huge": 0, "wgrad_side_stream": False,
                   "deterministic": True})
    rt.apply()
    assert options.OPTS.bconv_fp4 is False
    assert options.OPTS.tile_huge == 0
    assert options.OPTS.wgrad_side_stream is False
    assert options.OPTS.deterministic is True
    d = rt.as_dict()
    assert d["graph"] == "off" and d["force_dp"] is False and d["tile_huge"] == 0


def test_runtime_rejects_bad_graph_mode():
    rt = Runtime()
    with pytest.raises(ValueError, match="runtime.graph"):
        configure(rt, {"graph": "sometimes"})


def test_set_options_rejects_unknown_names():
    with pytest.raises(TypeError, match="unknown kernel option"):
        options.set_options(not_a_switch=1)


def test_runtime_is_part_of_the_experiment_config():
    from typing import Tuple

    from zookeeper_amd.core.component import component
    from zookeeper_amd.core.field import ComponentField, Field
    from zookeeper_amd.data import PadCropAndFlip, SyntheticCIFAR10
    from zookeeper_amd.models import BinaryNet
    from zookeeper_amd.train import Adam, TrainingExperiment

    @component
    class Exp(TrainingExperiment):
        dataset = ComponentField(SyntheticCIFAR10)
        input_shape: Tuple[int, int, int] = Field((32, 32, 3))
        preprocessing = ComponentField(PadCropAndFlip, pad_size=40)
        model = ComponentField(BinaryNet)
        optimizer = ComponentField(Adam)
        epochs = Field(1)
        batch_size = Field(8)

    exp = Exp()
    configure(exp, {"runtime.stem_fused": False, "runtime.graph": "auto"})
    flat = flatten_config(exp)
    assert flat["runtime.stem_fused"] is False
    assert flat["runtime.graph"] == "auto"
    assert "runtime.deterministic" in flat


_DEBUG_ONLY = {"ZK_NATIVE", "ZK_DEBUG_SYNC", "ZK_DEBUG_SYNC_LOG", "ZK_DEBUG_STEM",
               "ZK_COMM_DEBUG_EVENTS"}


def test_ops_and_kernels_read_no_runtime_environment():
    """Only debugging hooks may read the environment under ops/ and csrc/."""
    found = set()
    for sub in ("ops", "csrc"):
        for dirpath, _, files in os.walk(os.path.join(ROOT, "zookeeper_amd", sub)):
            for fn in files:
                if not fn.endswith((".py", ".hip", ".cpp", ".h")) or fn == "build.py":
                    continue
                src = open(os.path.join(dirpath, fn)).read()
                found |= set(re.findall(r'(?:environ\.get|getenv)\(\s*"([A-Z_0-9]+)"', src))
                found |= set(re.findall(r'environ\[\s*"([A-Z_0-9]+)"', src))
    assert found <= _DEBUG_ONLY, found - _DEBUG_ONLY


def test_visible_gpu_count_from_env_and_sysfs(tmp_path):
    for i, gid in enumerate([0, 1234, 5678]):  # node 0 is the CPU
        d = tmp_path / str(i)
        d.mkdir()
        (d / "gpu_id").write_text(f"{gid}\n")
    root = str(tmp_path)
    assert visible_gpu_count({}, root) == 2
    assert visible_gpu_ids({}, root) == ["0", "1"]
    assert visible_gpu_count({"HIP_VISIBLE_DEVICES": "1"}, root) == 1
    assert visible_gpu_count({"HIP_VISIBLE_DEVICES": ""}, root) == 0
    # faked ids on a host without GPUs (CPU rehearsals of 8-GPU sweeps)
    fake = {"HIP_VISIBLE_DEVICES": "0,1,2,3,4,5,6,7"}
    assert visible_gpu_count(fake, str(tmp_path / "none")) == 8
    assert visible_gpu_ids(fake, root) == [str(i) for i in range(8)]


def test_hw_queues_default_and_user_override(monkeypatch):
    """bench.py / dist.init raise the process to 16 hardware queues (HIP's
    default 4, which the boxes export explicitly, serialised the comm
    stream's waits with the input copies); ZK_HW_QUEUES picks a value, and a
    larger user setting stays."""
    from zookeeper_amd.parallel.devices import HW_QUEUES, configure_hw_queues

    monkeypatch.delenv("ZK_HW_QUEUES", raising=False)
    monkeypatch.delenv("GPU_MAX_HW_QUEUES", raising=False)
    assert configure_hw_queues() == str(HW_QUEUES) == "16"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    assert configure_hw_queues() == "16"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "24")
    assert configure_hw_queues() == "24"
    monkeypatch.setenv("ZK_HW_QUEUES", "6")
    assert configure_hw_queues() == "6"
