"""A tiny @task used by the sweep / launcher tests."""

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from zookeeper_amd import Field, cli, task  # noqa: E402


@task
class RecordConfig:
    lr: float = Field(0.1)
    wd: float = Field(0.0)
    fail_if_lr: float = Field(-1.0)
    out_dir: str = Field(".")

    def run(self):
        if self.lr == self.fail_if_lr:
            raise SystemExit(5)
        rec = {"lr": self.lr, "wd": self.wd,
               "hip_visible": os.environ.get("HIP_VISIBLE_DEVICES"),
               "rank": os.environ.get("RANK"), "world": os.environ.get("WORLD_SIZE")}
        name = f"lr{self.lr}_wd{self.wd}_r{os.environ.get('RANK', '0')}.json"
        with open(os.path.join(self.out_dir, name), "w") as f:
            json.dump(rec, f)


if __name__ == "__main__":
    cli()
