"""Data parallelism on the GPU training path.

* Two ranks on the box's one GPU (gloo transport; RCCL wants a GPU per
  rank): the HIP kernels' direct gradients must reach the bucketed
  all-reduce, the initial broadcast must align the replicas, and identical
  per-rank data must give the single-process result.
* One rank with a 1-rank RCCL (``nccl``) communicator and the bucketer
  forced on: the exact code path of the 8-GPU run -- comm-stream
  ``all_reduce`` on device tensors, ``work.wait()`` ordering against
  ProcessGroupNCCL's stream, timing events -- must reproduce the run without
  data parallelism and time every step's collectives."""

import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
WORKER = os.path.join(os.path.dirname(HERE), "dp_gpu_worker.py")


def _run(mode, out, nproc, side="1", graph="0", force="0", backend="gloo", rt="",
         check_order="0", comm="auto", prio="0", extra=None):
    """The worker in the shipped communicator settings by default
    (``runtime.comm_backend="auto"``, ``comm_high_priority=False``)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4", ZK_TEST_SIDE=side,
               ZK_TEST_GRAPH=graph, ZK_TEST_FORCE_DP=force, ZK_TEST_BACKEND=backend,
               ZK_TEST_RT=rt, ZK_TEST_CHECK_ORDER=check_order, ZK_TEST_COMM=comm,
               ZK_TEST_COMM_PRIO=prio, **(extra or {}))
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    if nproc == 1:
        return subprocess.run([sys.executable, WORKER, mode, str(out)], env=env,
                              timeout=240).returncode
    from zookeeper_amd.parallel.launch import spawn

    return spawn([sys.executable, WORKER, mode, str(out)], nproc, env=env)


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")


# Stated run-to-run tolerance of the parameters after the worker's SGD steps
# (relative L2) for a run that is not bit-reproducible; every mode of the
# framework now is (fixed-order split-K, BN and loss sums; grid-rounded fp64
# BN statistics), so the tests below hold both modes to atol = rtol = 0.
DEFAULT_MODE_REL = 1e-4


def _close(a, b, exact):
    if exact:
        torch.testing.assert_close(a, b, atol=0, rtol=0)
    else:
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < DEFAULT_MODE_REL, rel


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["deterministic", "default"])
@pytest.mark.parametrize("side,graph", [("1", "0"), ("0", "0"), ("1", "1")],
                         ids=["side-stream", "single-stream", "graph"])
def test_two_ranks_match_single_process_on_same_data(tmp_path, side, graph, mode):
    """Deterministic mode: two ranks on the same batches average identical
    gradients (g + g = 2g, times 1/2, is exact in fp32), so the result must
    equal the single-process run bit for bit.  The default mode is
    gradient-reproducible too since round 4 (slab split-K, fixed-order BN and
    loss sums), so it must match bit for bit as well."""
    exact = True
    rt = "deterministic=1" if mode == "deterministic" else ""
    assert _run("same", tmp_path, 1, side, graph, rt=rt) == 0
    assert _run("same", tmp_path, 2, side, graph, rt=rt) == 0
    ref = torch.load(tmp_path / "same_w1_r0.pt", weights_only=True)
    r0 = torch.load(tmp_path / "same_w2_r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "same_w2_r1.pt", weights_only=True)
    assert r0["buckets"] > 1
    assert r0["graph"] == (graph == "1") and ref["graph"] == (graph == "1")
    assert r0["comm_steps"] == 2  # every step's collectives were timed
    _close(r0["params"], r1["params"], exact)
    torch.testing.assert_close(r0["init"], ref["init"], atol=0, rtol=0)
    assert (ref["params"] - ref["init"]).norm().item() > 0
    _close(r0["params"], ref["params"], exact)


@pytest.mark.timeout(300)
def test_two_ranks_disjoint_data_stay_identical(tmp_path):
    """Also the bucket-order debug check (runtime.check_bucket_order) with
    side-stream weight gradients on: both ranks launch the same bucket
    sequence every step, and the cross-rank comparison ran every step."""
    assert _run("split", tmp_path, 2, side="1", check_order="1") == 0
    r0 = torch.load(tmp_path / "split_w2_r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "split_w2_r1.pt", weights_only=True)
    torch.testing.assert_close(r0["params"], r1["params"], atol=0, rtol=0)
    assert r0["loss"] == r0["loss"] and r1["loss"] == r1["loss"]  # finite
    assert r0["order_checks"] == r1["order_checks"] == 2
    assert r0["last_order"] == r1["last_order"]
    assert sorted(r0["last_order"]) == list(range(r0["buckets"]))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["deterministic", "default"])
@pytest.mark.parametrize("side,graph", [("1", "0"), ("0", "0"), ("1", "1")],
                         ids=["side-stream", "single-stream", "graph"])
def test_rccl_single_rank_forced_dp_matches_plain_run(tmp_path, side, graph, mode):
    """The shipped transport (``runtime.comm_backend="auto"``: the in-tree
    RCCL communicator after its agreed set-up and canary) with a 1-rank
    ``nccl`` group and the bucketer forced on: the forced run must equal the
    plain run BIT FOR BIT in the deterministic AND the default mode (every
    gradient sum is fixed-order since round 4; round 3's default mode used
    fp32 atomics whose noise the binary blocks amplified:
    profiles/r3/g_dp_forced_diag.md).  Under graph replay the collectives are
    captured with the backward."""
    rt = "deterministic=1" if mode == "deterministic" else ""
    assert _run("same", tmp_path, 1, side, graph, rt=rt) == 0
    assert _run("same", tmp_path, 1, side, graph, force="1", backend="nccl", rt=rt) == 0
    ref = torch.load(tmp_path / "same_w1_r0.pt", weights_only=True)
    dp = torch.load(tmp_path / "same_w1dp_r0.pt", weights_only=True)
    assert dp["backend"] == "nccl" and dp["bucketer"] and not ref["bucketer"]
    assert dp["native"]  # "auto" selected the native communicator
    assert dp["buckets"] > 1
    assert dp["graph"] == (graph == "1")
    if graph == "0":
        # pop_timings: one record per step, with real (non-negative) spans
        assert dp["comm_steps"] == 2, dp["timings"]
        for t in dp["timings"]:
            assert t["comm_ms"] >= 0 and t["bucket_sum_ms"] >= 0 and t["exposed_ms"] >= 0
    torch.testing.assert_close(dp["init"], ref["init"], atol=0, rtol=0)
    assert (ref["params"] - ref["init"]).norm().item() > 0
    # a 1-rank all-reduce is the identity and nothing else differs
    torch.testing.assert_close(dp["params"], ref["params"], atol=0, rtol=0)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("side,graph", [("1", "0"), ("1", "1")], ids=["side-stream", "graph"])
def test_process_group_transport_forced_dp_matches_plain_run(tmp_path, side, graph):
    """``runtime.comm_backend="torch"`` (ProcessGroupNCCL work objects, the
    fallback of "auto"), default mode: bit-equal to the plain run."""
    assert _run("same", tmp_path, 1, side, graph) == 0
    assert _run("same", tmp_path, 1, side, graph, force="1", backend="nccl", comm="torch") == 0
    ref = torch.load(tmp_path / "same_w1_r0.pt", weights_only=True)
    dp = torch.load(tmp_path / "same_w1dp_r0.pt", weights_only=True)
    assert dp["bucketer"] and not dp["native"]
    assert dp["comm_steps"] == 2, dp["timings"]
    torch.testing.assert_close(dp["params"], ref["params"], atol=0, rtol=0)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("graph", ["0", "1"], ids=["eager", "graph"])
def test_native_rccl_communicator_forced_dp_matches_plain_run(tmp_path, graph):
    """runtime.comm_backend="native" (no fallback), default mode, high-priority
    comm stream: bit-equal to the plain run."""
    assert _run("same", tmp_path, 1, "1", graph) == 0
    assert _run("same", tmp_path, 1, "1", graph, force="1", backend="nccl",
                comm="native", prio="1") == 0
    ref = torch.load(tmp_path / "same_w1_r0.pt", weights_only=True)
    dp = torch.load(tmp_path / "same_w1dp_r0.pt", weights_only=True)
    assert dp["native"] and dp["bucketer"]
    assert dp["graph"] == (graph == "1")
    torch.testing.assert_close(dp["params"], ref["params"], atol=0, rtol=0)


@pytest.mark.timeout(300)
def test_aborted_communicator_is_not_replayed(tmp_path):
    """after the watchdog marks the native communicator failed,
    the next graph step raises BEFORE replaying the captured collectives
    (their RCCL resources are freed by the abort)."""
    assert _run("same", tmp_path, 1, "1", "1", force="1", backend="nccl",
                extra={"ZK_TEST_ABORT_AFTER": "2", "ZK_TEST_STEPS": "4"}) == 0
    res = torch.load(tmp_path / "abort.pt", weights_only=True)
    assert res["raised"] is True and res["replays"] == 0, res
