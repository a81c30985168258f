"""Sweep launcher, --nproc launcher and the experiment CLI end to end (CPU)."""

import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
TASK = os.path.join(HERE, "sweep_task.py")


def _env(**kw):
    e = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", **kw)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "HIP_VISIBLE_DEVICES"):
        e.pop(k, None)
    e.update(kw)
    return e


def test_grid_parsing():
    from zookeeper_amd.sweep import expand, parse_grid, run_name

    axes = parse_grid(["lr=[0.1,0.01]", "optimizer.wd=[0,1e-4,2e-4]", "name=['a']"])
    combos = expand(axes)
    assert len(combos) == 6
    assert combos[0] == {"lr": 0.1, "optimizer.wd": 0, "name": "a"}
    assert run_name({"optimizer.wd": 1e-4, "lr": 0.1}) == "optimizer-wd_0.0001__lr_0.1"


@pytest.mark.timeout(300)
def test_sweep_runs_grid_concurrently(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    cmd = [sys.executable, TASK, "RecordConfig", f"out_dir={str(out)!r}",
           "--grid", "lr=[0.1,0.2]", "--grid", "wd=[0.0,0.5]", "--max-parallel", "2"]
    env = _env(ZK_SWEEP_DIR=str(tmp_path / "sweep"), HIP_VISIBLE_DEVICES="0,1,2,3")
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stdout + res.stderr
    recs = [json.load(open(out / f)) for f in sorted(os.listdir(out))]
    assert sorted((r["lr"], r["wd"]) for r in recs) == [(0.1, 0.0), (0.1, 0.5), (0.2, 0.0), (0.2, 0.5)]
    # each run saw exactly one (its own) GPU
    assert all(len(r["hip_visible"].split(",")) == 1 for r in recs)
    summary = json.load(open(tmp_path / "sweep" / "sweep.json"))
    assert len(summary) == 4 and all(s["exit_code"] == 0 for s in summary)


@pytest.mark.timeout(300)
def test_sweep_packs_runs_per_gpu(tmp_path):
    out = tmp_path / "out"
    out.mkdir()
    cmd = [sys.executable, TASK, "RecordConfig", f"out_dir={str(out)!r}",
           "--grid", "lr=[0.1,0.2]", "--grid", "wd=[0.0,0.5]", "--runs-per-gpu", "2"]
    env = _env(ZK_SWEEP_DIR=str(tmp_path / "sweep"), HIP_VISIBLE_DEVICES="4,5")
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stdout + res.stderr
    recs = [json.load(open(out / f)) for f in sorted(os.listdir(out))]
    assert len(recs) == 4
    # two GPUs x two runs each: every run on one GPU, each GPU used twice
    assert sorted(r["hip_visible"] for r in recs) == ["4", "4", "5", "5"]
    assert res.stdout.count("[sweep] start") == 4
    # all four slots filled before any run finished
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("[sweep]")]
    assert all(ln.startswith("[sweep] start") for ln in lines[:4]), lines


def test_sweep_slots_round_robin(monkeypatch, tmp_path):
    from zookeeper_amd import sweep

    started, run_ids = [], []

    class FakeProc:
        def __init__(self, argv, env, stdout, stderr):
            started.append(env.get("HIP_VISIBLE_DEVICES"))
            run_ids.append(env["ZK_RUN_ID"])

        def poll(self):
            return 0

    monkeypatch.setattr(sweep.subprocess, "Popen", FakeProc)
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    rc = sweep.run_sweep(["x"], [("lr", [1, 2, 3, 4, 5, 6])], gpus_per_run=2,
                         sweep_dir=str(tmp_path), poll_s=0.0, runs_per_gpu=3)
    assert rc == 0
    assert started == ["0,1", "2,3", "0,1", "2,3", "0,1", "2,3"]
    assert run_ids == [f"lr_{i}" for i in range(1, 7)]


@pytest.mark.timeout(300)
def test_sweep_reports_failed_runs(tmp_path):
    cmd = [sys.executable, TASK, "RecordConfig", f"out_dir={str(tmp_path)!r}", "fail_if_lr=0.2",
           "--grid", "lr=[0.1,0.2]"]
    env = _env(ZK_SWEEP_DIR=str(tmp_path / "sweep"))
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 1
    summary = {s["name"]: s["exit_code"] for s in json.load(open(tmp_path / "sweep" / "sweep.json"))}
    assert summary == {"lr_0.1": 0, "lr_0.2": 5}


@pytest.mark.timeout(300)
def test_nproc_launches_ranks(tmp_path):
    cmd = [sys.executable, TASK, "RecordConfig", f"out_dir={str(tmp_path)!r}", "--nproc", "2"]
    res = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr
    recs = [json.load(open(tmp_path / f)) for f in sorted(os.listdir(tmp_path))]
    assert sorted(r["rank"] for r in recs) == ["0", "1"]
    assert all(r["world"] == "2" for r in recs)


@pytest.mark.timeout(600)
def test_example_smoke_epochs_zero():
    """The reference CI smoke run: `larq_experiment.py BinaryNetMnist epochs=0`."""
    res = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "larq_experiment.py"),
                          "BinaryNetMnist", "epochs=0"], env=_env(), capture_output=True,
                         text=True, timeout=500)
    assert res.returncode == 0, res.stderr[-2000:]
    assert "BinaryNetMnist(" in res.stdout


@pytest.mark.timeout(900)
def test_training_checkpoint_and_resume(tmp_path):
    base = [sys.executable, os.path.join(ROOT, "examples", "larq_experiment.py"), "BinaryNetMnist",
            "batch_size=8", "steps_per_epoch=2", "validate=False", "print_summary=False",
            f"output_dir={str(tmp_path)!r}", "model.filters=32", "model.dense_units=64",
            "dataset.num_train_examples=64"]
    res = subprocess.run(base + ["epochs=1"], env=_env(), capture_output=True, text=True,
                         timeout=600)
    assert res.returncode == 0, res.stderr[-2000:]
    run_dir = tmp_path / "BinaryNetMnist" / "run"
    assert (run_dir / "checkpoints" / "step_00000002" / "model.pt").exists()
    rec = json.load(open(run_dir / "config.json"))
    cfg = rec["config"]
    # the resolved dotted-key config, replayable through configure / the CLI
    assert rec["task"] == "BinaryNetMnist"
    assert cfg["batch_size"] == 8 and cfg["steps_per_epoch"] == 2
    assert cfg["model"] == "BinaryNet" and cfg["model.filters"] == 32
    assert cfg["dataset"] == "SyntheticMNIST" and cfg["dataset.num_train_examples"] == 64
    assert cfg["preprocessing.pad_size"] == 32
    assert cfg["metrics"] == ["accuracy"]
    assert "BinaryNetMnist(" in rec["tree"]
    lines = open(run_dir / "metrics.jsonl").read().strip().splitlines()
    assert json.loads(lines[-1])["step"] == 2
    res = subprocess.run(base + ["epochs=2"], env=_env(), capture_output=True, text=True,
                         timeout=600)
    assert res.returncode == 0, res.stderr[-2000:]
    assert "resumed from" in res.stdout
    assert (run_dir / "checkpoints" / "step_00000004").exists()


@pytest.mark.timeout(900)
def test_cifar10_binarynet_task_runs_on_cpu(tmp_path):
    """BASELINE.json config 4: the CIFAR-10 BinaryNet @task end to end on the
    CPU (world_size 1): trains, validates, checkpoints, logs metrics."""
    cmd = [sys.executable, os.path.join(ROOT, "examples", "larq_experiment.py"), "BinaryNetCifar10",
           "epochs=1", "batch_size=8", "steps_per_epoch=3", "print_summary=False",
           f"output_dir={str(tmp_path)!r}", "model.filters=32", "model.dense_units=64",
           "dataset.num_train_examples=64", "dataset.num_validation_examples=16",
           "metrics=['accuracy','sparse_top_k_categorical_accuracy']"]
    res = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=800)
    assert res.returncode == 0, res.stderr[-2000:]
    run_dir = tmp_path / "BinaryNetCifar10" / "run"
    lines = open(run_dir / "metrics.jsonl").read().strip().splitlines()
    recs = [json.loads(line) for line in lines]
    assert any(r.get("step") == 3 for r in recs)
    # configured Keras-style metrics: top-1 and top-5 logged per flush
    assert all("top1" in r and "top5" in r for r in recs)
    assert all(r["top5"] >= r["top1"] for r in recs)
    assert "val_top5=" in res.stdout
    assert (run_dir / "checkpoints" / "step_00000003" / "model.pt").exists()


@pytest.mark.timeout(600)
def test_sweep_records_throughput_and_loss(tmp_path):
    """BASELINE config 5's record: each run of a training sweep reports its
    images/sec and final loss in sweep.json (via ZK_RESULT_JSON)."""
    cmd = [sys.executable, os.path.join(ROOT, "examples", "larq_experiment.py"), "BinaryNetCifar10",
           "epochs=1", "batch_size=8", "steps_per_epoch=2", "print_summary=False", "validate=False",
           "model.filters=32", "model.dense_units=64", "dataset.num_train_examples=64",
           "--grid", "learning_rate=[0.001,0.01]"]
    env = _env(ZK_SWEEP_DIR=str(tmp_path / "sweep"))
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=560)
    assert res.returncode == 0, res.stdout[-2000:] + res.stderr[-2000:]
    summary = json.load(open(tmp_path / "sweep" / "sweep.json"))
    assert sorted(s["name"] for s in summary) == ["learning_rate_0.001", "learning_rate_0.01"]
    for s in summary:
        assert s["exit_code"] == 0 and s["steps"] == 2
        assert s["images_per_sec"] > 0
        assert s["final_loss"] == s["final_loss"] and s["final_loss"] > 0  # finite


@pytest.mark.timeout(600)
def test_config5_grid_dp2_runs_on_disjoint_device_pairs(tmp_path):
    """BASELINE config 5, rehearsed on the CPU: an lr x wd grid of four
    TrainingExperiment runs across 8 (faked) GPUs, each run data-parallel on
    its own pair (--gpus-per-run 2 -> every run relaunched as 2 ranks over
    gloo).  All four runs start before any finishes, each writes
    result.json, and sweep.json carries per-run images/sec and final loss."""
    sweep_dir = tmp_path / "sweep"
    cmd = [sys.executable, os.path.join(ROOT, "examples", "train_imagenet.py"), "TrainImageNet",
           "--grid", "learning_rate=[1e-3,2e-3]", "--grid", "optimizer.weight_decay=[0.0,5e-5]",
           "--gpus-per-run", "2",
           "model=BinaryNet", "model.filters=16", "model.dense_units=64",
           "input_shape=(32,32,3)", "dataset.image_shape=(32,32,3)", "dataset.num_classes=10",
           "dataset.num_train_examples=64", "dataset.num_validation_examples=0",
           "batch_size=4", "steps_per_epoch=3", "epochs=1", "log_every=1", "print_summary=False"]
    env = _env(ZK_SWEEP_DIR=str(sweep_dir), HIP_VISIBLE_DEVICES="0,1,2,3,4,5,6,7",
               ZK_DIST_TIMEOUT_S="240")
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=560)
    assert res.returncode == 0, res.stdout[-4000:] + res.stderr[-4000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("[sweep]")]
    starts = [ln for ln in lines if ln.startswith("[sweep] start")]
    assert len(starts) == 4
    assert all(ln.startswith("[sweep] start") for ln in lines[:4]), lines  # concurrent
    pairs = sorted(ln.split("devices ")[1] for ln in starts)
    assert pairs == ["['0', '1']", "['2', '3']", "['4', '5']", "['6', '7']"], pairs
    summary = json.load(open(sweep_dir / "sweep.json"))
    assert len(summary) == 4
    for rec in summary:
        assert rec["exit_code"] == 0, rec
        assert len(rec["devices"]) == 2
        assert rec["images_per_sec"] > 0 and rec["final_loss"] == rec["final_loss"]
        assert os.path.exists(sweep_dir / rec["name"] / "result.json")
        log = open(sweep_dir / rec["name"] / "stdout.log").read()
        assert "world" in log or rec["steps"] == 3
    grid = sorted((r["overrides"]["learning_rate"], r["overrides"]["optimizer.weight_decay"])
                  for r in summary)
    assert grid == [("0.001", "0.0"), ("0.001", "5e-05"), ("0.002", "0.0"), ("0.002", "5e-05")]
