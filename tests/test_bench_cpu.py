"""``bench.py`` launch contract on CPU (gloo): ``--gpus N`` without a
``WORLD_SIZE`` spawns N ranks itself and prints ONE JSON line (rank 0) with
``n_gpus == N``; a ``WORLD_SIZE`` that disagrees with ``--gpus`` is an error,
never a silent 1-rank run."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
ARGS = ["--steps", "2", "--warmup", "1", "--batch", "2", "--image-size", "32"]


def _env():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "OMP_NUM_THREADS"):
        env.pop(k, None)
    return env


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_self_spawns_ranks(n):
    res = subprocess.run([sys.executable, BENCH, "--gpus", str(n), *ARGS], env=_env(),
                         capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = _json_lines(res.stdout)
    assert len(lines) == 1, res.stdout  # rank 0 only
    rec = lines[0]
    assert rec["n_gpus"] == n
    assert rec["config"]["parallelism"] == f"dp{n}"
    assert rec["config"]["global_batch"] == 2 * n
    assert rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["higher_is_better"] is True
    # a gloo/CPU rehearsal never carries the bare headline metric string
    assert rec["metric"].startswith("rehearsal")
    assert rec["config"]["dist_backend"] == "gloo"
    # the driver-timed default streams data through the host pipeline, and
    # the communicator set-up is recorded
    assert rec["config"]["data_path"] == "stream"
    comm = rec["config"]["comm"]
    assert comm["bucket_mb"] == 10.0 and sum(comm["bucket_sizes_mb"]) > 0
    for k in ("comm_high_priority", "rccl_min_channels", "rccl_max_channels", "cpu_affinity",
              "check_bucket_order"):
        assert k in rec["config"]["runtime"]


@pytest.mark.timeout(120)
def test_bench_world_mismatch_is_an_error():
    env = _env()
    env["WORLD_SIZE"] = "1"
    res = subprocess.run([sys.executable, BENCH, "--gpus", "2", *ARGS], env=env,
                         capture_output=True, text=True, timeout=100, cwd=ROOT)
    assert res.returncode == 2
    assert "WORLD_SIZE" in res.stderr
    assert not _json_lines(res.stdout)


@pytest.mark.timeout(200)
def test_bench_single_rank_json_contract():
    res = subprocess.run([sys.executable, BENCH, *ARGS], env=_env(), capture_output=True,
                         text=True, timeout=180, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    (rec,) = _json_lines(res.stdout)
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert key in rec
    assert rec["n_gpus"] == 1 and rec["scaling"] == "weak"
    for key in ("model", "global_batch", "seq_len", "parallelism"):
        assert key in rec["config"]


@pytest.mark.timeout(200)
def test_bench_force_dp_single_rank_runs_the_bucketer():
    """``--force-dp``: one rank, but the bucketed all-reduce path is on (a
    1-rank process group; gloo here, RCCL on a GPU)."""
    res = subprocess.run([sys.executable, BENCH, *ARGS, "--force-dp", "--rt", "tile_huge=0"],
                         env=_env(), capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-3000:]
    (rec,) = _json_lines(res.stdout)
    assert rec["n_gpus"] == 1
    assert rec["config"]["buckets"] >= 1
    assert rec["config"]["runtime"]["force_dp"] is True
    assert rec["config"]["runtime"]["tile_huge"] == 0
