"""Shared pytest configuration.

* ``gpu`` marker: tests that need a real MI355X (run with ``-m gpu`` on the
  GPU box); everything else must pass on a CPU-only host.
* ``clean_cli`` fixture: @task registers commands on the process-global click
  group, so tests that define tasks restore the registry afterwards.
"""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (gfx950)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture
def clean_cli():
    from zookeeper_amd.core.cli import cli

    saved = dict(cli.commands)
    cli.commands = {}
    try:
        yield cli
    finally:
        cli.commands = saved
