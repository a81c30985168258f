"""Config-layer overheads, the only quantities SURVEY.md §6 could measure on
the reference (CPU, 8 vCPU): ``import`` time, ``configure`` of an
experiment-sized tree (3 sub-components, 18 fields) plus first touches,
cached / first field access, cached ``@factory``-built field access.

    python tools/bench_config.py [--json out.json]

The tree mirrors the reference's test fixtures
(zookeeper/core/component_test.py) and its example
(examples/larq_experiment.py:106-153): a task-like root with dataset,
preprocessing and model children, scoped inheritance of ``num_classes`` /
``input_shape`` from the root, and a factory-built optimizer field.
"""

import argparse
import json
import os
import subprocess
import sys
import time
from typing import Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def import_ms(reps: int = 5) -> float:
    code = ("import time,sys; sys.path.insert(0, %r); t=time.perf_counter(); "
            "import zookeeper_amd; print((time.perf_counter()-t)*1e3)" % ROOT)
    vals = []
    for _ in range(reps):
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                             check=True).stdout
        vals.append(float(out.strip().splitlines()[-1]))
    return sorted(vals)[len(vals) // 2]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    args = ap.parse_args()

    from zookeeper_amd import ComponentField, Field, component, configure, factory

    @component
    class Data:
        name: str = Field("mnist")
        train_split: str = Field("train")
        validation_split: str = Field("test")
        num_classes: int = Field(10)
        shuffle: bool = Field(True)

    @component
    class Prep:
        input_shape: Tuple[int, int, int] = Field()
        pad_size: int = Field(4)
        flip: bool = Field(True)

    @component
    class Net:
        num_classes: int = Field()
        input_shape: Tuple[int, int, int] = Field()
        filters: int = Field(128)
        dense_units: int = Field(1024)
        kernel_size: int = Field(3)

    class Opt:
        def __init__(self, lr):
            self.lr = lr

    @factory
    class OptFactory:
        learning_rate: float = Field()

        def build(self) -> Opt:
            return Opt(self.learning_rate)

    @component
    class Exp:
        dataset: Data = ComponentField(Data)
        preprocessing: Prep = ComponentField(Prep)
        model: Net = ComponentField(Net)
        optimizer: Opt = ComponentField(OptFactory)
        input_shape: Tuple[int, int, int] = Field((28, 28, 1))
        num_classes: int = Field(10)
        epochs: int = Field(100)
        batch_size: int = Field(128)
        learning_rate: float = Field(5e-3)

    conf = {"epochs": 3, "model.filters": 64, "dataset.shuffle": False}

    def configure_and_touch():
        e = Exp()
        configure(e, conf)
        e.model.num_classes, e.model.input_shape, e.preprocessing.input_shape
        e.dataset.name, e.optimizer
        return e

    for _ in range(200):
        configure_and_touch()
    n = 2000
    t = time.perf_counter()
    for _ in range(n):
        configure_and_touch()
    cfg_us = (time.perf_counter() - t) / n * 1e6

    e = configure_and_touch()
    m = e.model
    m.filters
    n = 200000
    t = time.perf_counter()
    for _ in range(n):
        m.filters
    cached_us = (time.perf_counter() - t) / n * 1e6

    class Plain:
        filters = 64
    p = Plain()
    t = time.perf_counter()
    for _ in range(n):
        p.filters
    plain_ns = (time.perf_counter() - t) / n * 1e9

    t = time.perf_counter()
    for _ in range(n):
        e.optimizer
    factory_us = (time.perf_counter() - t) / n * 1e6

    # first access: a fresh configured tree each time, one inherited field
    trees = []
    for _ in range(3000):
        x = Exp()
        configure(x, conf)
        trees.append(x.model)
    t = time.perf_counter()
    for mm in trees:
        mm.num_classes
    first_us = (time.perf_counter() - t) / len(trees) * 1e6

    res = {
        "import_ms": round(import_ms(), 2),
        "configure_tree_plus_first_touches_us": round(cfg_us, 2),
        "cached_field_access_us": round(cached_us, 3),
        "plain_attribute_ns": round(plain_ns, 1),
        "first_field_access_inherited_us": round(first_us, 3),
        "cached_factory_field_access_us": round(factory_us, 3),
        "reference_survey_s6": {"import_ms": 28, "configure_tree_plus_first_touches_us": "95-133",
                                "cached_field_access_us": 1.34, "plain_attribute_ns": 39,
                                "first_field_access_us": 6.6,
                                "cached_factory_field_access_us": 2.7},
    }
    print(json.dumps(res, indent=2))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=2)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
