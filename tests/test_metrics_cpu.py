"""Configurable metrics (Keras ``compile(metrics=...)`` names,
examples/larq_experiment.py:118) and the resolved-config run record."""

import pytest
import torch

from zookeeper_amd.train.metrics import MetricsLogger, resolve_metrics, topk_hits


def test_resolve_metric_names():
    m = resolve_metrics(["accuracy", "sparse_top_k_categorical_accuracy", "top3", "loss"])
    assert list(m) == ["top1", "top5", "top3"]
    assert m["top1"] is None and callable(m["top5"]) and callable(m["top3"])
    assert resolve_metrics(["sparse_categorical_accuracy"]) == {"top1": None}
    with pytest.raises(ValueError, match="Unknown metric 'auc'"):
        resolve_metrics(["auc"])


def test_topk_hits_matches_definition():
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(64, 10, generator=g)
    labels = torch.randint(0, 10, (64,), generator=g)
    for k in (1, 3, 5, 10, 20):
        ref = sum(int(labels[i] in logits[i].argsort(descending=True)[:k]) for i in range(64))
        assert int(topk_hits(k)(logits, labels)) == ref


def test_logger_records_configured_metrics(tmp_path):
    log = MetricsLogger(torch.device("cpu"), str(tmp_path / "m.jsonl"), echo=False,
                        metrics=["accuracy", "top5"])
    log.update(torch.tensor(2.0), torch.tensor(3), 8, {"top5": torch.tensor(6)})
    log.update(torch.tensor(1.0), torch.tensor(1), 8, {"top5": torch.tensor(7)})
    rec = log.flush(2)
    assert rec["loss"] == pytest.approx(1.5)
    assert rec["top1"] == pytest.approx(4 / 16)
    assert rec["top5"] == pytest.approx(13 / 16)


def test_flatten_config_roundtrip():
    from typing import Tuple

    from zookeeper_amd import ComponentField, Field, component, configure
    from zookeeper_amd.core.component import flatten_config

    @component
    class Child:
        a: int = Field(1)
        shared: float = Field()

    @component
    class Other(Child):
        pass

    @component
    class Parent:
        shared: float = Field(0.5)
        shape: Tuple[int, int] = Field((2, 3))
        child: Child = ComponentField(Child)
        name: str = Field("x")

    p = Parent()
    configure(p, {"child": "Other", "child.a": 7, "name": "run"})
    flat = flatten_config(p)
    assert flat == {"shared": 0.5, "shape": (2, 3), "child": "Other", "child.a": 7,
                    "name": "run"}  # child.shared is inherited: recorded once
    q = Parent()
    configure(q, {k: v for k, v in flat.items()})
    assert flatten_config(q) == flat
